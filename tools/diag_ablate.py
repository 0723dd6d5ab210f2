"""In-pipeline time of each kernel family by graph ablation (sacx_time_graph)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "sac-expert_amd"))
import bench  # noqa: E402

cfgd = bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "hc"]
import torch  # noqa: E402
from sac_eo.common.seeding import derive_seeds  # noqa: E402
seeds = {k: int(v[0]) for k, v in derive_seeds(0, 1).items()}
eng = bench.build_engine(cfgd, seeds, torch.device("cuda", 0))
eng.step(256)
eng.sync()
out = {"full_us": eng.time_graph(10) * 1e3}
for fam in ("k_rng", "k_gemm", "k_actor_head", "k_qhead", "k_actor_bwd"):
    out[fam] = out["full_us"] - eng.time_graph(10, fam) * 1e3
print(json.dumps({k: round(v, 2) for k, v in out.items()}))
