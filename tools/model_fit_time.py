"""World-model fit (A16) timing: µs per model-fit step (2 models x minibatch 200) at the bench
configs' shapes, graph replay and eager.  usage: python tools/model_fit_time.py [config] [steps]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "sac-expert_amd"))
import bench  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "hc_eo"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 512
from sac_eo.common.seeding import derive_seeds  # noqa: E402
import torch  # noqa: E402

cfgd = dict(bench.CONFIGS[cfg], buffer=200_000)
sd = {k: int(v[0]) for k, v in derive_seeds(0, 1).items()}
eng = bench.build_engine(cfgd, sd, device=torch.device("cuda", 0))
mb = eng.cfg.model_batch
idx = np.random.RandomState(3).randint(cfgd["buffer"], size=(n + 64, 2, mb)).astype(np.int32)
for mode in (("graph",) if os.environ.get("MFT_GRAPH_ONLY") else ("graph", "eager", "graph")):
    eng.model_fit(idx[:64], eager=(mode == "eager"))
    eng.sync()
    t0 = time.perf_counter()
    eng.model_fit(idx[64:], eager=(mode == "eager"))
    eng.sync()
    us = (time.perf_counter() - t0) / n * 1e6
    S, A, Hm = cfgd["S"], cfgd["A"], 512
    macs = 3 * ((S + A) * Hm + Hm * Hm + Hm * (S + 1)) - (S + A) * Hm
    print(f"{cfg} model fit ({mode}): {us:.2f} us/step = {2.0 * macs * 2 * mb / us / 1e6:.2f} TFLOP/s; "
          f"last loss {eng.model_stats(1)[0]}", flush=True)
eng.close()
