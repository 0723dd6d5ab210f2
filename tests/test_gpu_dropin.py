"""The drop-in loop's speculative sampler.  In the reference's cadence (act -> _update -> env.step
-> add, /root/reference/sac_eo/algs/SAC_expert.py:779-797) act_host queues the next update's
randint + normals right behind the action kernel, for the ring as it is then, and the following
step(1) replays the sampler-less graph on them when the ring still has that size; any other
draw from the global stream (a stochastic action, get_state) or an append in between first
undoes it.  Whatever the interleaving, the run must equal the same calls with the speculation
off (SACX_SPEC=0), bit for bit: losses, weights, Adam state, ring and the RNG stream."""
import numpy as np
import pytest

from helpers import load_learner, make_learner

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("full,tui", [(False, 1), (True, 1), (False, 2)])
def test_speculative_sampler_equals_plain(gpu_available, monkeypatch, full, tui):
    """tui = 2: the Polyak gate reads num_timesteps, which the speculative steps leave to the
    control block when it already holds the value (k_set_ctl skipped); the timesteps jump now and
    then, so a stale value would gate the wrong updates."""
    from sac_eo.engine import Engine, EngineConfig
    B, N, n = 64, 600, 48
    outs, hits = [], []
    for spec in ("1", "0"):
        monkeypatch.setenv("SACX_SPEC", spec)
        ocfg, st, buf, nrm, _ = make_learner(act="relu", B=B, N=N, seed=5, done_p=0.05)
        cap = N if full else N + 200          # full: every append drops the oldest row
        eng = Engine(EngineConfig(s_dim=17, a_dim=6, activation="relu", batch=B, buffer_capacity=cap, graph_steps=1,
                                  target_update_int=tui))
        load_learner(eng, st, buf, nrm, None, 0.1)
        eng.rng_set_state(np.random.RandomState(12).get_state())
        rs = np.random.RandomState(3)
        for j in range(n):
            o, o2 = rs.normal(size=17).astype(np.float32), rs.normal(size=17).astype(np.float32)
            a = eng.act_host(o, deterministic=(j % 11 != 7))     # now and then a stochastic action
            late = j % 9 == 4                                     # now and then the add before the update
            if late:
                eng.append(o[None], a[None], np.array([0.5], np.float32), o2[None], np.zeros(1, np.float32))
            eng.step(1, num_timesteps=j + j // 7, ts_increment=1)
            if j % 13 == 5:
                eng.append(np.stack([o, o2]), np.stack([a, a]), np.zeros(2), np.stack([o2, o]), np.zeros(2))  # 2 rows
            elif not late:
                eng.append(o[None], a[None], np.array([0.5], np.float32), o2[None], np.zeros(1, np.float32))
            if j == 30:
                eng.rng_get_state()                               # an observation point mid-run
            if j == 40:
                assert np.isfinite(eng.stats(1)).all()            # another one
        eng.sync()
        hits.append(eng.spec_hits())
        outs.append((eng.stats(n).copy(), eng.v["params"].cpu().numpy().copy(), eng.v["adam_v"].cpu().numpy().copy(),
                     eng.v["replay"].cpu().numpy().copy(), eng.rng_get_state()[1].copy(), eng.ctl()["cur_size"]))
        eng.close()
    assert hits[1] == 0 and hits[0] >= n // 2, hits          # the speculative path did run
    for i, (a, b) in enumerate(zip(*outs)):
        assert np.array_equal(a, b), i


def test_speculative_sac_eo_with_deferred_alpha(gpu_available, monkeypatch):
    """SAC-EO (two world models, expert permutations) through the same cadence, with the
    things that must run a deferred alpha branch first: a new expert set / epsilon mid-run
    (alpha.final mixes the expert MSE with it), a multi-update step, a stats read."""
    from helpers import make_pair
    n, outs, hits = 40, [], []
    for spec in ("1", "0"):
        monkeypatch.setenv("SACX_SPEC", spec)
        eng, ocfg, st, buf, nrm, expert = make_pair(act="relu", B=64, N=800, seed=8, use_expert=True,
                                                    graph_steps=1, done_p=0.05)
        eng.rng_set_state(np.random.RandomState(21).get_state())
        rp = np.random.RandomState(4)
        eng.push_perms(np.stack([rp.permutation(eng.cfg.expert_batch) for _ in range(n + 8)]))
        rs = np.random.RandomState(5)
        t = 0
        for j in range(n):
            o, o2 = rs.normal(size=17).astype(np.float32), rs.normal(size=17).astype(np.float32)
            a = eng.act_host(o, deterministic=(j % 7 != 3))
            eng.step(1, num_timesteps=t, ts_increment=1)
            t += 1
            eng.append(o[None], a[None], np.array([0.25], np.float32), o2[None], np.zeros(1, np.float32))
            if j == 15:
                eng.set_expert(expert["s"], expert["sp"], 0.3)
            if j == 25:
                eng.step(3, num_timesteps=t, ts_increment=1)
                t += 3
            if j == 33:
                assert np.isfinite(eng.stats(1)).all()
        eng.sync()
        hits.append(eng.spec_hits())
        outs.append((eng.stats(n + 3).copy(), eng.v["params"].cpu().numpy().copy(),
                     eng.v["adam_m"].cpu().numpy().copy(), eng.rng_get_state()[1].copy(),
                     {k: v for k, v in eng.ctl().items() if k in ("t_sac", "num_timesteps", "cur_size", "start", "step_seq")}))
        eng.close()
    assert hits[1] == 0 and hits[0] >= n // 2, hits
    for i, (a, b) in enumerate(zip(*outs)):
        if isinstance(a, dict):
            assert a == b, (a, b)
        else:
            assert np.array_equal(a, b), i


@pytest.mark.parametrize("use_expert", [False, True])
def test_speculative_packed_lockstep(gpu_available, monkeypatch, use_expert):
    """The lock-step --runs cadence on a packed handle (act_host_seeds -> step(1) ->
    append_host_seeds; single_seed_plan): every seed's speculative draw and deferred alpha branch
    == the same calls with SACX_SPEC=0, bit for bit, incl. a stochastic round and a per-seed
    observation (SeedView stats) mid-run."""
    from sac_eo.engine import Engine, EngineConfig
    K, B, N, n = 3, 64, 700, 30
    outs, hits = [], []
    for spec in ("1", "0"):
        monkeypatch.setenv("SACX_SPEC", spec)
        learners = [make_learner(act="relu", B=B, N=N, seed=40 + 3 * k, use_expert=use_expert, done_p=0.05)
                    for k in range(K)]
        eng = Engine(EngineConfig(s_dim=17, a_dim=6, activation="relu", batch=B, buffer_capacity=N + 100,
                                  graph_steps=1, seeds=K, single_seed_plan=True, use_expert=use_expert,
                                  expert_capacity=20, expert_batch=20, epsilon=0.1))
        for k, (ocfg, st, buf, nrm, expert) in enumerate(learners):
            eng.select_seed(k)
            load_learner(eng, st, buf, nrm, expert, 0.1)
            eng.rng_set_state(np.random.RandomState(50 + k).get_state())
            if use_expert:
                rp = np.random.RandomState(60 + k)
                eng.push_perms(np.stack([rp.permutation(20) for _ in range(n + 4)]))
        eng.select_seed(0)
        rs = np.random.RandomState(9)
        for j in range(n):
            o = rs.normal(size=(K, 17)).astype(np.float32)
            o2 = rs.normal(size=(K, 17)).astype(np.float32)
            a = eng.act_host_seeds(o, deterministic=(j % 9 != 4))
            eng.step(1, num_timesteps=j, ts_increment=1)
            eng.append_host_seeds(o[:, None], a[:, None], np.full((K, 1), 0.5, np.float32), o2[:, None],
                                  np.zeros((K, 1), np.float32))
            if j == 17:
                assert np.isfinite(eng.seed_view(1).stats(1)).all()
        eng.sync()
        hits.append(eng.spec_hits())
        res = []
        for k in range(K):
            eng.select_seed(k)
            res += [eng.stats(n).copy(), eng.v["params"].cpu().numpy().copy(), eng.rng_get_state()[1].copy()]
        outs.append(res)
        eng.close()
    assert hits[1] == 0 and hits[0] >= n // 2, hits
    for i, (a, b) in enumerate(zip(*outs)):
        assert np.array_equal(a, b), i


def test_speculative_packed_per_seed_act(gpu_available, monkeypatch):
    """A per-seed act_host on a packed handle (select_seed(k), act_host(det)) followed by a packed
    step(1): the speculative draw it queues must cover EVERY seed's stream (not only the selected
    seed's), so the run equals the same calls with SACX_SPEC=0 bit for bit, seeds 1..K-1 included."""
    from sac_eo.engine import Engine, EngineConfig
    K, B, N, n = 3, 64, 700, 24
    outs, hits = [], []
    for spec in ("1", "0"):
        monkeypatch.setenv("SACX_SPEC", spec)
        learners = [make_learner(act="relu", B=B, N=N, seed=70 + 3 * k, done_p=0.05) for k in range(K)]
        eng = Engine(EngineConfig(s_dim=17, a_dim=6, activation="relu", batch=B, buffer_capacity=N + 100,
                                  graph_steps=1, seeds=K, single_seed_plan=True))
        for k, (ocfg, st, buf, nrm, expert) in enumerate(learners):
            eng.select_seed(k)
            load_learner(eng, st, buf, nrm, expert, 0.1)
            eng.rng_set_state(np.random.RandomState(80 + k).get_state())
        rs = np.random.RandomState(11)
        for j in range(n):
            eng.select_seed(j % K)
            o = rs.normal(size=17).astype(np.float32)
            eng.act_host(o, deterministic=(j % 7 != 3))
            eng.step(1, num_timesteps=j, ts_increment=1)
        eng.sync()
        hits.append(eng.spec_hits())
        res = []
        for k in range(K):
            eng.select_seed(k)
            res += [eng.stats(n).copy(), eng.v["params"].cpu().numpy().copy(), eng.rng_get_state()[1].copy()]
        outs.append(res)
        eng.close()
    assert hits[1] == 0 and hits[0] >= n // 2, hits
    for i, (a, b) in enumerate(zip(*outs)):
        assert np.array_equal(a, b), i


def test_held_append_and_skipped_ctl_observed(gpu_available, monkeypatch):
    """The drop-in cadence's held 1-row append (it runs inside the next act's launch) and the
    skipped k_set_ctl must be invisible: right after an append_host the ring read through Engine.v
    holds the row; any other entry point (a multi-update step, a stochastic act, a 2-row append,
    get_state) queues the held row first; ts_increment changes force the control block's rewrite.
    The gather's polar workgroups (SACX_SPEC_POLAR) and the pinned completion counts in place of
    event markers (SACX_APP_CTR) likewise.  The whole run equals SACX_APP_DEFER=0 SACX_CTL_SKIP=0
    SACX_SPEC_POLAR=0 SACX_APP_CTR=0 bit for bit."""
    from sac_eo.engine import Engine, EngineConfig
    B, N, n = 64, 500, 40
    outs = []
    for opt in ("1", "0"):
        for var in ("SACX_APP_DEFER", "SACX_CTL_SKIP", "SACX_SPEC_POLAR", "SACX_APP_CTR"):
            monkeypatch.setenv(var, opt)
        _, st, buf, nrm, _ = make_learner(act="relu", B=B, N=N, seed=6, done_p=0.05)
        eng = Engine(EngineConfig(s_dim=17, a_dim=6, activation="relu", batch=B, buffer_capacity=N + 100,
                                  graph_steps=1, target_update_int=3))
        load_learner(eng, st, buf, nrm, None, 0.1)
        eng.rng_set_state(np.random.RandomState(31).get_state())
        rs = np.random.RandomState(9)
        t, inc = 0, 1
        for j in range(n):
            o, o2 = rs.normal(size=17).astype(np.float32), rs.normal(size=17).astype(np.float32)
            a = eng.act_host(o, deterministic=(j % 13 != 6))
            if j == 20:
                inc = 2                                       # a new ts_increment: the control block is rewritten
            eng.step(1, num_timesteps=t, ts_increment=inc)
            t += inc
            r = np.array([0.1 * j], np.float32)
            eng.append(o[None], a[None], r, o2[None], np.zeros(1, np.float32))
            if j % 9 == 4:                                    # the held row is visible at once
                c = eng.ctl()
                row = eng.v["replay"][(c["start"] + c["cur_size"] - 1) % (N + 100)].cpu().numpy()
                assert row[2 * 17 + 6] == r[0] and np.array_equal(row[:17], o)
            if j == 14:
                eng.step(2, num_timesteps=t, ts_increment=inc)
                t += 2 * inc
            if j == 27:
                eng.append(np.stack([o2, o]), np.stack([a, a]), np.zeros(2), np.stack([o, o2]), np.zeros(2))
            if j == 33:
                eng.rng_get_state()
        eng.sync()
        outs.append((eng.stats(n + 2).copy(), eng.v["params"].cpu().numpy().copy(), eng.v["adam_v"].cpu().numpy().copy(),
                     eng.v["replay"].cpu().numpy().copy(), eng.rng_get_state()[1].copy(),
                     {k: v for k, v in eng.ctl().items() if k in ("t_sac", "num_timesteps", "cur_size", "start", "step_seq")}))
        eng.close()
    for i, (x, y) in enumerate(zip(*outs)):
        if isinstance(x, dict):
            assert x == y, (x, y)
        else:
            assert np.array_equal(x, y), i
