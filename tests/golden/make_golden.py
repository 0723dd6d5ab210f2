"""Generates the committed golden fixtures under tests/golden/.

rng_golden.npz   -- outputs of NumPy's legacy np.random.RandomState (the
                    reference's RNG: sac_eo/common/buffers.py:136,
                    sac_eo/actors/continuous_actors.py:351) for fixed seeds:
                    randint(high, 256) for several highs and normal((256, 6)).
sac_golden.npz   -- a short fp64 oracle trajectory (tiny shapes) with the
                    randoms drawn in the reference order, used to detect
                    regressions of the oracle itself and as the small-size
                    device parity case.

Run:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import sac_oracle as O  # noqa: E402

SEEDS = [0, 2773201285, 2590541744]
HIGHS = [777, 5000, 2 ** 20, 10 ** 6, 4 * 10 ** 6]


def make_rng():
    out = {"highs": np.array(HIGHS, np.int64)}
    for seed in SEEDS:
        for high in HIGHS:
            out[f"seed_{seed}_int_{high}"] = np.random.RandomState(seed).randint(high, size=256)
        out[f"seed_{seed}_normal"] = np.random.RandomState(seed).normal(size=(256, 6))
    # a full step's worth of draws in the reference order from the known-answer
    # expert seed (train.py:101 makes it the global stream origin)
    rs = np.random.RandomState(2590541744)
    R = O.draw_step_randoms(rs, 10 ** 6, 256, 6)
    for k, v in R.items():
        out["step_" + k] = v
    np.savez_compressed(os.path.join(HERE, "rng_golden.npz"), **out)


SAC_RNG_SEED = 11     # global MT19937 stream of the trajectory
SAC_STEPS = 10


def sac_inputs():
    """The golden trajectory's inputs: (cfg, fp32 initial state, buffer, normalisers)."""
    cfg = O.Config(S=5, A=2, hidden=(16, 16), act="tanh", B=16)
    st = O.init_state(cfg, seed=1, bias_scale=0.05)
    rs = np.random.RandomState(0)
    N = 64
    buf = dict(s=rs.normal(size=(N, 5)).astype(np.float32),
               a=rs.uniform(-1, 1, (N, 2)).astype(np.float32),
               sp=rs.normal(size=(N, 5)).astype(np.float32),
               r=rs.normal(size=N).astype(np.float32),
               d=(rs.uniform(size=N) < 0.1).astype(np.float64))
    return cfg, st, buf, O.Normalizers.identity(5, 2)


def make_sac():
    cfg, st, buf, nrm = sac_inputs()
    st = st.astype(np.float64)
    N = buf["r"].shape[0]
    g = np.random.RandomState(SAC_RNG_SEED)
    losses = []
    for _ in range(SAC_STEPS):
        R = O.draw_step_randoms(g, N, cfg.B, cfg.A)
        n = [O.f32_noise(R[k]) for k in ("noise_t", "noise_pi", "noise_alpha")]
        stt = O.sac_update(st, cfg, nrm, O.gather(buf, R["idx"]), *n)
        losses.append([stt["q1_loss"], stt["q2_loss"], stt["p_loss"], stt["alpha_loss"], stt["alpha"]])
    out = dict(buf_s=buf["s"], buf_a=buf["a"], buf_sp=buf["sp"], buf_r=buf["r"], buf_d=buf["d"],
               losses=np.array(losses))
    for i, w in enumerate(st.actor):
        out[f"actor_{i}"] = w
    for k in range(2):
        for i, w in enumerate(st.q[k]):
            out[f"q{k}_{i}"] = w
            out[f"t{k}_{i}"] = st.q_targ[k][i]
    out["logstd"] = st.logstd
    out["alpha"] = st.alpha
    np.savez_compressed(os.path.join(HERE, "sac_golden.npz"), **out)


if __name__ == "__main__":
    make_rng()
    make_sac()
    print("wrote", os.listdir(HERE))
