"""Multi-rank data-parallel mode (config C4) on ONE GPU: the in-process reduce.

Two libsacx handles are ranks 0 and 1 of one data-parallel group (sacx_dp_init_local): each
samples B/2 rows from its own replay ring with its own stream, stores its local gradients, and
at each of the update's three all-reduce points (critic range, actor range + logstd, alpha) one
kernel sums the two ranks' gradient ranges and writes the sum back to both -- what RCCL's
ncclAllReduce(sum) does across GPUs; the plans, local-gradient stores and Adam-apply launches are
the RCCL mode's own.  Checked against tests/test_dp.py's protocol on the fp64 oracle:

* the two ranks stay bit-identical to each other (weights, targets, alpha, Adam moments);
* they equal the single learner's update on the concatenated B-row batch (indices and noise
  drawn from the two ranks' streams), within the single-learner tolerance.
"""
import numpy as np
import pytest
import torch

import sac_oracle as O
from helpers import load_learner, make_learner, relerr

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("act", ["relu", "tanh"])
def test_dp_two_local_ranks_equal_global_batch(gpu_available, act):
    from sac_eo.engine import Engine, EngineConfig
    B, steps, N, eps = 128, 24, 4000, 0.1
    ocfg, st, buf, nrm, _ = make_learner(act=act, B=B, N=N, seed=71, done_p=0.02)
    st64 = st.astype(np.float64)
    stream = torch.cuda.current_stream()
    engs = []
    for r in range(2):
        cfg = EngineConfig(s_dim=17, a_dim=6, activation=act, batch=B // 2, buffer_capacity=N, graph_steps=8)
        e = Engine(cfg, stream=stream, dp_local=(2, r))
        load_learner(e, st, buf, nrm, None, eps)
        engs.append(e)
    rss = [np.random.RandomState(900 + r) for r in range(2)]
    for r, e in enumerate(engs):
        e.rng_set_state(rss[r].get_state())
    ref = []
    for t in range(steps):
        Rs = [O.draw_step_randoms(rs, N, B // 2, ocfg.A) for rs in rss]
        batch = [np.concatenate(x) for x in zip(*(O.gather(buf, R["idx"]) for R in Rs))]
        noise = [O.f32_noise(np.concatenate([R[k] for R in Rs])) for k in ("noise_t", "noise_pi", "noise_alpha")]
        o = O.sac_update(st64, ocfg, nrm, batch, *noise)
        ref.append([o["q1_loss"], o["q2_loss"], o["alpha"]])
    Engine.dp_local_step(engs, steps, num_timesteps=0, ts_increment=1)
    for e in engs:
        e.sync()
    # the ranks are replicas, bit for bit
    for seg in ("params", "adam_m", "adam_v"):
        assert np.array_equal(engs[0].v[seg].cpu().numpy(), engs[1].v[seg].cpu().numpy()), seg
    # and equal the global-batch learner
    worst = 0.0
    for name, nets in (("actor", st64.actor), ("q0", st64.q[0]), ("q1", st64.q[1]), ("t0", st64.q_targ[0]),
                       ("t1", st64.q_targ[1])):
        for a, b in zip(engs[0].get_net(name), nets):
            worst = max(worst, relerr(a, b))
    assert abs(engs[0].alpha() - float(st64.alpha)) <= 1e-6 * max(abs(float(st64.alpha)), 1e-5)
    s0, s1 = engs[0].stats(steps), engs[1].stats(steps)
    q_dev = 0.5 * (s0[:, :2].astype(np.float64) + s1[:, :2])       # mean of the two local means
    ref = np.array(ref)
    q_err = relerr(q_dev, ref[:, :2])
    print(f"{act}: weights worst {worst:.2e}, Q losses {q_err:.2e} over {steps} updates")
    assert worst < 1e-4 and q_err < 1e-4, (worst, q_err)
    for e in engs:
        e.close()


def test_dp_rccl_two_processes(gpu_available):
    """Config C4 over RCCL between two fresh processes (bench.py --mode dpcheck --gpus 2: one GPU per
    rank, ncclAllReduce inside the captured update graph): the ranks' parameters and Adam state
    bit-identical after 64 updates, and equal to the single learner's updates on the concatenated
    batches.  RCCL refuses two ranks on one device, so a one-GPU box skips."""
    import json
    import os
    import subprocess
    import sys
    if torch.cuda.device_count() < 2:
        pytest.skip("RCCL data-parallel ranks need one GPU each: fewer than 2 visible")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--mode", "dpcheck", "--gpus", "2"],
                         capture_output=True, text=True, timeout=400, env=env, cwd=root)
    assert out.returncode == 0, out.stderr[-2000:]
    res = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])["dp_c4"]
    print(res)
    assert res["ranks"] == 2 and res["rccl_world_size"] == 2
    assert res["dp_ranks_identical"] and res["matches_single_learner"], res
