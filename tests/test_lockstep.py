"""The lock-step driver (sac_eo.algs.lockstep) on CPU with stand-in learners and a stand-in
packed engine: one batched call per round of identical requests, results routed back in seed
order, and a clear error when the learners' schedules diverge."""
import numpy as np
import pytest

from sac_eo.algs.lockstep import run_lockstep


class FakeEngine:
    def __init__(self, seeds):
        self.seeds = seeds
        self.calls = []

    def act_host_seeds(self, obs, deterministic):
        self.calls.append(("act", obs.shape, deterministic))
        return obs[:, :2] * 2.0

    def step(self, n, num_timesteps, ts_increment):
        self.calls.append(("update", n, num_timesteps, ts_increment))

    def append_host_seeds(self, s, a, r, sp, d):
        self.calls.append(("add", s.shape))
        return s.shape[1]


class FakeLearner:
    def __init__(self, k, steps, g_every):
        self.k, self.steps, self.g_every = k, steps, g_every
        self.seen = []

    def _train_loop(self, total, params):
        for t in range(self.steps):
            obs = np.full(4, self.k + t, np.float32)
            a = yield ("act", obs, True)
            self.seen.append(a.copy())
            if t % self.g_every == 0:
                yield ("update", 3, t, 0)
            n = yield ("add", (obs[None], a[None], np.zeros(1), obs[None], np.zeros(1), np.zeros(1)))
            assert n == 1
        return f"run{self.k}"


def test_lockstep_rounds_and_routing():
    eng = FakeEngine(3)
    algs = [FakeLearner(k, 5, 2) for k in range(3)]
    assert run_lockstep(algs, eng, 5, [None] * 3) == ["run0", "run1", "run2"]
    assert [c[0] for c in eng.calls].count("act") == 5 and [c[0] for c in eng.calls].count("update") == 3
    for k, alg in enumerate(algs):                 # each learner got its own row's action
        assert [float(x[0]) for x in alg.seen] == [2.0 * (k + t) for t in range(5)]


def test_lockstep_divergence_raises():
    eng = FakeEngine(2)
    algs = [FakeLearner(0, 5, 2), FakeLearner(1, 5, 3)]      # different update schedules
    with pytest.raises(RuntimeError, match="diverged"):
        run_lockstep(algs, eng, 5, [None] * 2)
    eng = FakeEngine(2)
    with pytest.raises(RuntimeError, match="diverged"):
        run_lockstep([FakeLearner(0, 4, 2), FakeLearner(1, 5, 2)], eng, 5, [None] * 2)
