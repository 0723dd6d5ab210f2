"""The committed SAC golden trajectory (tests/golden/sac_golden.npz, written by
tests/golden/make_golden.py): 10 updates of a tiny tanh learner (S=5, A=2, 16x16, B=16)
with the reference-order randoms of RandomState(11).

CPU: the oracle still reproduces the fixture (a regression pin of the checker).
GPU: the device update chain, started from the same state, buffer and stream, lands on
the fixture's losses and final weights (rel 1e-4 of each tensor's max; fp32 device vs
the fp64 oracle trajectory)."""
import os
import sys

import numpy as np
import pytest

import sac_oracle as O

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
import make_golden as G  # noqa: E402

FIX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "sac_golden.npz")


def _fixture():
    with np.load(FIX) as z:
        return {k: z[k] for k in z.files}


def test_oracle_reproduces_sac_golden():
    fx = _fixture()
    cfg, st, buf, nrm = G.sac_inputs()
    for k in ("s", "a", "sp", "r", "d"):
        assert np.array_equal(buf[k], fx["buf_" + k])
    st = st.astype(np.float64)
    g = np.random.RandomState(G.SAC_RNG_SEED)
    losses = []
    for _ in range(G.SAC_STEPS):
        R = O.draw_step_randoms(g, buf["r"].shape[0], cfg.B, cfg.A)
        n = [O.f32_noise(R[k]) for k in ("noise_t", "noise_pi", "noise_alpha")]
        o = O.sac_update(st, cfg, nrm, O.gather(buf, R["idx"]), *n)
        losses.append([o["q1_loss"], o["q2_loss"], o["p_loss"], o["alpha_loss"], o["alpha"]])
    np.testing.assert_allclose(np.array(losses), fx["losses"], rtol=1e-9, atol=1e-12)
    for i, w in enumerate(st.actor):
        np.testing.assert_allclose(w, fx[f"actor_{i}"], rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(st.alpha, fx["alpha"], rtol=1e-9)


@pytest.mark.gpu
@pytest.mark.parametrize("eager", [True, False])
def test_device_matches_sac_golden(gpu_available, eager):
    from sac_eo.engine import Engine, EngineConfig
    from helpers import load_learner
    fx = _fixture()
    cfg, st, buf, nrm = G.sac_inputs()
    N = buf["r"].shape[0]
    eng = Engine(EngineConfig(s_dim=cfg.S, a_dim=cfg.A, hidden=cfg.hidden, activation="tanh", batch=cfg.B,
                              buffer_capacity=N, graph_steps=4))
    load_learner(eng, st, buf, nrm, None, 0.0)
    eng.rng_set_state(np.random.RandomState(G.SAC_RNG_SEED).get_state())
    eng.step(G.SAC_STEPS, num_timesteps=0, ts_increment=1, eager=eager)
    eng.sync()
    dev = eng.stats(G.SAC_STEPS)
    ref = fx["losses"]
    # q1, q2, p losses, alpha loss, alpha
    for col in range(5):
        rel = np.abs(dev[:, col] - ref[:, col]) / np.maximum(np.abs(ref[:, col]), 1e-6)
        assert rel.max() < 1e-4, (col, rel.max())
    got = eng.get_net("actor")
    for i in range(len(got)):
        w = fx[f"actor_{i}"]
        assert np.max(np.abs(got[i] - w)) / np.max(np.abs(w)) < 1e-4, i
    for k in range(2):
        gq, gt = eng.get_net(f"q{k}"), eng.get_net(f"t{k}")
        for i in range(len(gq)):
            for got_w, key in ((gq[i], f"q{k}_{i}"), (gt[i], f"t{k}_{i}")):
                w = fx[key]
                assert np.max(np.abs(got_w - w)) / np.max(np.abs(w)) < 1e-4, key
    eng.close()
