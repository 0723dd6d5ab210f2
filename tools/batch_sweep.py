"""Experiment: updates/s of one learner vs batch size (HC shapes), a proxy for how much
work a launch of the update chain absorbs before its duration grows."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "sac-expert_amd"))
import torch  # noqa: E402,F401
import bench  # noqa: E402
from sac_eo.common.seeding import derive_seeds  # noqa: E402

cfgd = dict(bench.CONFIGS[os.environ.get("BS_CONFIG", "hc")])
seeds = {k: int(v[0]) for k, v in derive_seeds(0).items()}
for B in [int(x) for x in sys.argv[1:]]:
    e = bench.build_engine(cfgd, seeds, device=torch.device("cuda:0"), batch=B)
    e.step(256)
    e.sync()
    t0 = time.perf_counter()
    e.step(1024)
    e.sync()
    el = time.perf_counter() - t0
    print(f"B={B} updates/s={1024 / el:.1f} us={el / 1024 * 1e6:.2f}", flush=True)
    e.close()
