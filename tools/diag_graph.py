"""Diagnostic: one config under several launch modes vs the oracle and vs eager."""
import os, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "sac-expert_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import numpy as np
import sac_oracle as O
from helpers import make_pair, oracle_step

mode = sys.argv[1]            # eager | g1 | g8
act, B, seed, done = sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), float(sys.argv[5])
steps = int(sys.argv[6]) if len(sys.argv) > 6 else 8
gs = 1 if mode == "g1" else 8
eng, ocfg, st, buf, nrm, ex = make_pair(act=act, B=B, seed=seed, done_p=done, graph_steps=gs)
N = buf["r"].shape[0]
rs = np.random.RandomState(123)
eng.rng_set_state(rs.get_state())
Rs = [O.draw_step_randoms(rs, N, B, ocfg.A) for _ in range(steps)]
eng.step(steps, eager=(mode == "eager"))
eng.sync()
dev = eng.stats(steps)
ref = [oracle_step(st, ocfg, nrm, buf, R) for R in Rs]
out = {"mode": mode, "fork": os.environ.get("SACX_NO_FORK") is None, "cfg": [act, B, seed, done]}
out["rel_q"] = [[float(abs(dev[i, k] - ref[i][n]) / abs(ref[i][n])) for k, n in ((0, "q1_loss"), (1, "q2_loss"))] for i in range(min(4, steps))]
out["dev_q"] = dev[:3, :2].tolist()
out["ref_q"] = [[ref[i]["q1_loss"], ref[i]["q2_loss"]] for i in range(3)]
out["params_sum"] = float(eng.v["params"].double().sum().item())
out["Hq2_slab_sums"] = [float(x) for x in eng.v["ws.Hq2"].double().reshape(4, B, -1).sum(dim=(1, 2)).tolist()]
print(json.dumps(out))
