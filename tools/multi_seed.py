"""Packed seeds: K independent learners in one handle (cfg.seeds = K, one launch chain with
grid z = seed) vs one learner.  Prints aggregate and per-seed updates/s.

usage: MS_CONFIG=hc python tools/multi_seed.py [K ...]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "sac-expert_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from sac_eo.common.seeding import derive_seeds  # noqa: E402


def run(K, steps=1024, warmup=256, config="hc"):
    cfgd = dict(bench.CONFIGS[config])
    cfgd["buffer"] = int(os.environ.get("MS_BUFFER", cfgd["buffer"]))
    ds = derive_seeds(0, runs=K)
    seeds = [{n: int(v[k]) for n, v in ds.items()} for k in range(K)]
    eng = bench.build_engine(cfgd, seeds, device=torch.device("cuda:0"))
    eng.step(warmup)
    eng.sync()
    t0 = time.perf_counter()
    eng.step(steps)
    eng.sync()
    el = time.perf_counter() - t0
    ok = True
    for k in range(K):
        eng.select_seed(k)
        ok = ok and bool(np.all(np.isfinite(eng.stats(1)[0])))
    eng.close()
    return K * steps / el, el / steps * 1e6, ok


if __name__ == "__main__":
    Ks = [int(x) for x in sys.argv[1:]] or [1, 2, 4]
    cfg = os.environ.get("MS_CONFIG", "hc")
    for K in Ks:
        v, us, ok = run(K, config=cfg)
        print(f"config={cfg} K={K} aggregate={v:.1f} updates/s per_seed={v / K:.1f} "
              f"us_per_round={us:.2f} finite={ok}", flush=True)
