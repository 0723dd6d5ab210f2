"""Where does the device's alpha trajectory leave the fp64 oracle's?  (tests/test_gpu_schedule.py
setup: 300 updates at graph_steps = 128.)  Prints per update alpha (device, fp64, fp32 oracle),
the oracle's alpha Adam m and the policy-loss errors around the first divergence."""
import sys
sys.path[:0] = ["tests", "oracle", "sac-expert_amd"]
import numpy as np
import sac_oracle as O
from helpers import make_pair, oracle_step

use_expert = len(sys.argv) > 1 and sys.argv[1] == "eo"
B, steps = 256, 300
eng, ocfg, st, buf, nrm, expert = make_pair(act="relu", B=B, seed=13, use_expert=use_expert, done_p=0.01, graph_steps=128)
st32 = st.astype(np.float32)
N = buf["r"].shape[0]
rs = np.random.RandomState(321)
gen = np.random.default_rng(78)
eng.rng_set_state(rs.get_state())
Rs = [O.draw_step_randoms(rs, N, B, ocfg.A, n_expert=20 if use_expert else 0, gen=gen) for _ in range(steps)]
if use_expert:
    eng.push_perms(np.stack([R["perm"] for R in Rs]))
rows = []
for part in (100, 200):
    eng.step(part, num_timesteps=len(rows), ts_increment=1)
    for R in Rs[len(rows):len(rows) + part]:
        o = oracle_step(st, ocfg, nrm, buf, R, expert)
        o32 = oracle_step(st32, ocfg, nrm, buf, R, expert)
        rows.append([float(st.alpha), float(st32.alpha), float(st.opt_alpha.m[0]), float(st32.opt_alpha.m[0]),
                     o["p_loss"], o32["p_loss"], o["alpha_loss"], o32["alpha_loss"], -o["alpha_loss"] / max(abs(float(st.alpha)), 1e-30)])
eng.sync()
dev = eng.stats(steps)
rows = np.array(rows)
first = None
for i in range(steps):
    if abs(dev[i, 4] - rows[i, 0]) > 1e-10 and first is None:
        first = i
print("first alpha divergence at update", first)
lo = max(0, (first or steps) - 5)
for i in range(lo, min(steps, lo + 40)):
    print(f"{i:4d} alpha dev {dev[i,4]:.9e} f64 {rows[i,0]:.9e} f32 {rows[i,1]:.9e} | m64 {rows[i,2]:+.3e} m32 {rows[i,3]:+.3e} "
          f"| p dev {dev[i,2]:.6e} f64 {rows[i,4]:.6e} | aloss dev {dev[i,3]:.4e} f64 {rows[i,6]:.4e}")
