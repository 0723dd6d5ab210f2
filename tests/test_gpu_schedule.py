"""Parity of the PRODUCTION schedule (graph_steps = 128, the bench's and EngineConfig's
default): the sampler runs ahead on a side stream and its slot ring (2 x SACX_NBATCH slots)
wraps many times inside one captured graph, so a slot-reuse race would show here and not in
the graph_steps = 8 tests.

* 300 updates (two 128-update graphs + one 44-update remainder graph) vs the fp64 oracle:
  Q1/Q2 losses and the policy loss (which carries SAC-EO's expert MSE, relative to the
  trajectory's scale) within 1e-4 over the first 100 updates (north_star) and TRAJ_TOL_300
  over all 300, weights / targets after 100 and 300 updates within PARAM_TOL_100 /
  PARAM_TOL_300 (norm-relative per tensor), the update sequence numbers and the RNG stream
  exact.
* graph replay == eager launches, bit for bit, at SACX_NBATCH 2 / 4 / 8 (± expert).
* 8 packed seeds at graph_steps = 128 == 8 one-seed engines, bit for bit.
Reference: SAC_exp._update (sac_eo/algs/SAC_expert.py:463-477), SAC._update (SAC.py:236-250).
"""
import numpy as np
import pytest

import sac_oracle as O
from helpers import load_learner, make_learner, make_pair, oracle_step

pytestmark = pytest.mark.gpu

PARAM_TOL_100 = 1e-4    # ||w_dev - w_oracle|| / ||w_oracle|| per tensor after 100 updates
PARAM_TOL_300 = 1e-2    # ... after 300 (fp32 vs fp64 rounding compounded through Adam)
TRAJ_TOL_300 = 3e-3     # Q / policy loss over all 300 updates (fp32 device vs fp64 oracle)


def _params_close(eng, st, use_expert):
    nets = [("actor", st.actor)] + [(f"q{k}", st.q[k]) for k in range(2)] + [(f"t{k}", st.q_targ[k]) for k in range(2)]
    worst = 0.0
    for name, ref in nets:
        for a, b in zip(eng.get_net(name), ref):
            worst = max(worst, float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)))
    return worst


@pytest.mark.parametrize("use_expert", [False, True])
def test_production_schedule_trajectory_300(gpu_available, use_expert):
    """step(100) (one 100-update graph) then step(200) (a 128-update graph + a 72-update one)."""
    B, steps = 256, 300
    eng, ocfg, st, buf, nrm, expert = make_pair(act="relu", B=B, seed=13, use_expert=use_expert, done_p=0.01,
                                                graph_steps=128)
    N = buf["r"].shape[0]
    rs = np.random.RandomState(321)
    gen = np.random.default_rng(78)
    eng.rng_set_state(rs.get_state())
    Rs = [O.draw_step_randoms(rs, N, B, ocfg.A, n_expert=20 if use_expert else 0, gen=gen) for _ in range(steps)]
    if use_expert:
        eng.push_perms(np.stack([R["perm"] for R in Rs]))
    ref = []
    for part in (100, 200):
        eng.prepare(part)
        eng.step(part, num_timesteps=len(ref), ts_increment=1)
        eng.sync()
        for R in Rs[len(ref):len(ref) + part]:
            o = oracle_step(st, ocfg, nrm, buf, R, expert)
            ref.append([o["q1_loss"], o["q2_loss"], o["p_loss"], o["alpha_loss"]])
        worst = _params_close(eng, st, use_expert)
        print(f"weights after {len(ref)} updates: worst ||dev - oracle|| / ||oracle|| per tensor {worst:.2e}")
        assert worst < (PARAM_TOL_100 if len(ref) == 100 else PARAM_TOL_300), (len(ref), worst)
    dev = eng.stats(steps)
    ref = np.array(ref)
    rel_q = np.abs(dev[:, :2] - ref[:, :2]) / np.abs(ref[:, :2])
    rel_p = np.abs(dev[:, 2] - ref[:, 2]) / np.max(np.abs(ref[:, 2]))
    # alpha loss relative to the trajectory's scale: once alpha sits at its 1e-5 clamp the loss
    # is ~1e-5 and its pointwise relative error says nothing
    rel_a = np.abs(dev[:, 3] - ref[:, 3]) / np.max(np.abs(ref[:, 3]))
    for lo in range(0, steps, 50):
        print(f"updates {lo}-{lo + 49}: q {rel_q[lo:lo + 50].max():.2e} p {rel_p[lo:lo + 50].max():.2e} "
              f"alpha {rel_a[lo:lo + 50].max():.2e}")
    # the north_star bar over the first 100 updates; beyond, fp32-vs-fp64 rounding compounds
    # through the Adam steps and alpha's clamp (a schedule fault -- a stale or overwritten
    # slot -- shows as 1e-2 to 1e-1 from the update it hits, see the slot-ring fix)
    assert rel_q[:100].max() < 1e-4, rel_q[:100].max()
    assert rel_p[:100].max() < 1e-4, rel_p[:100].max()
    assert rel_q.max() < TRAJ_TOL_300, rel_q.max()
    assert rel_p.max() < TRAJ_TOL_300, rel_p.max()
    assert rel_a.max() < 1e-3, rel_a.max()
    assert np.array_equal(dev[:, 7], np.arange(steps, dtype=np.float32))      # update sequence numbers
    got, exp = eng.rng_get_state(), rs.get_state()
    assert np.array_equal(got[1], exp[1]) and got[2] == exp[2] and got[3] == exp[3] and got[4] == exp[4]
    eng.close()


@pytest.mark.parametrize("nbatch,use_expert", [(2, False), (4, False), (8, False), (4, True), (8, True)])
def test_production_graph_equals_eager(gpu_available, monkeypatch, nbatch, use_expert):
    """graph_steps = 128, 300 updates: 2 full graphs + a 44-update remainder graph; the slot
    ring (2 * nbatch slots) wraps 16-64 times inside each graph."""
    monkeypatch.setenv("SACX_NBATCH", str(nbatch))
    n = 300
    outs = []
    for eager in (True, False):
        eng, *_ = make_pair(act="tanh", B=128, seed=22, use_expert=use_expert, graph_steps=128)
        eng.rng_set_state(np.random.RandomState(6).get_state())
        if use_expert:
            rs = np.random.RandomState(9)
            eng.push_perms(np.stack([rs.permutation(eng.cfg.expert_batch) for _ in range(n)]))
        eng.step(n, eager=eager)
        eng.sync()
        outs.append((eng.stats(n).copy(), eng.v["params"].cpu().numpy().copy(),
                     eng.v["adam_v"].cpu().numpy().copy(), eng.rng_get_state()[1].copy()))
        eng.close()
    for a, b in zip(*outs):
        assert np.array_equal(a, b)


def test_packed8_production_schedule(gpu_available, monkeypatch):
    """8 packed seeds (32x32 forward / dX tiles: 8 x 128 rows) at graph_steps = 128 over 150
    updates (a 128-update graph + a 22-update one) == 8 one-seed engines (16x16 tiles, eager)."""
    from sac_eo.engine import Engine, EngineConfig
    K, n, B, N, eps = 8, 150, 128, 3000, 0.1
    monkeypatch.setenv("SACX_FUSE_HEAD", "0")
    # the 32x32 plan keeps the separate actor head backward and the row-dot head; so do the
    # one-seed references (their folds would change the summation order)
    monkeypatch.setenv("SACX_FOLD_HBW", "0")
    monkeypatch.setenv("SACX_HEAD_PART", "0")
    learners = [make_learner(act="relu", B=B, N=N, seed=60 + 5 * k) for k in range(K)]

    def cfg(seeds, G):
        return EngineConfig(s_dim=17, a_dim=6, activation="relu", batch=B, buffer_capacity=N, graph_steps=G,
                            seeds=seeds)

    def drive(eng, k):
        _, st, buf, nrm, ex = learners[k]
        load_learner(eng, st, buf, nrm, ex, eps)
        eng.rng_set_state(np.random.RandomState(700 + k).get_state())

    packed = Engine(cfg(K, 128))
    for k in range(K):
        packed.select_seed(k)
        drive(packed, k)
    packed.select_seed(0)
    packed.step(n)
    packed.sync()
    got = []
    for k in range(K):
        packed.select_seed(k)
        got.append((packed.stats(n).copy(), packed.v["params"].cpu().numpy().copy(),
                    packed.v["adam_v"].cpu().numpy().copy(), packed.rng_get_state()[1].copy()))
    packed.close()
    monkeypatch.setenv("SACX_T32", "0")
    for k in range(K):
        e = Engine(cfg(1, 8))
        drive(e, k)
        e.step(n, eager=True)
        e.sync()
        ref = (e.stats(n), e.v["params"].cpu().numpy(), e.v["adam_v"].cpu().numpy(), e.rng_get_state()[1])
        e.close()
        for i, (a, b) in enumerate(zip(got[k], ref)):
            assert np.array_equal(a, b), (k, i)


def test_prepare_then_step_is_cached(gpu_available):
    """sacx_prepare(n) instantiates the graphs step(n) replays without running an update:
    the counters do not move, and the following step(n) equals an unprepared engine's."""
    outs = []
    for prep in (False, True):
        eng, *_ = make_pair(act="relu", B=64, seed=3, graph_steps=128)
        eng.rng_set_state(np.random.RandomState(2).get_state())
        if prep:
            eng.prepare(150)
            eng.sync()
            assert eng.ctl()["step_seq"] == 0
        eng.step(150)
        eng.sync()
        outs.append((eng.stats(150).copy(), eng.v["params"].cpu().numpy().copy()))
        eng.close()
    assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])
