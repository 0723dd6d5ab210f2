"""Full-state snapshot of a packed-seed handle (cfg.seeds = K): save_state writes every seed,
load_state restores every seed, and the resumed run is bit-identical for each of them."""
import numpy as np
import pytest

from helpers import load_learner, make_learner

pytestmark = pytest.mark.gpu


def test_packed_snapshot_resume(gpu_available, tmp_path):
    from sac_eo.engine import Engine, EngineConfig
    K, B, N = 3, 64, 2000
    learners = [make_learner(act="relu", B=B, N=N, seed=80 + k) for k in range(K)]

    def fresh():
        e = Engine(EngineConfig(s_dim=17, a_dim=6, batch=B, buffer_capacity=N, graph_steps=8, seeds=K))
        for k in range(K):
            e.select_seed(k)
            _, st, buf, nrm, ex = learners[k]
            load_learner(e, st, buf, nrm, ex, 0.1)
            e.rng_set_state(np.random.RandomState(30 + k).get_state())
        e.select_seed(0)
        return e

    def snap(e, n):
        out = []
        for k in range(K):
            e.select_seed(k)
            out.append((e.stats(n).copy(), e.v["params"].cpu().numpy().copy(), e.rng_get_state()[1].copy()))
        e.select_seed(0)
        return out

    eng = fresh()
    eng.step(9)
    eng.save_state(str(tmp_path / "snap"))
    eng.step(11)
    eng.sync()
    ref = snap(eng, 11)
    eng.close()
    eng2 = fresh()
    eng2.load_state(str(tmp_path / "snap"))
    eng2.step(11)
    eng2.sync()
    got = snap(eng2, 11)
    eng2.close()
    for k in range(K):
        for a, b in zip(ref[k], got[k]):
            assert np.array_equal(a, b), k
    assert not np.array_equal(ref[0][1], ref[1][1])
