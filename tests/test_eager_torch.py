"""The eager PyTorch-CPU baseline (oracle/sac_eager_torch.py, bench.py's reference-equivalent CPU
leg) computes the same update as the oracle: losses and every updated weight after two updates,
plain SAC and SAC-EO, and one world-model fit step (fp32 vs the fp64 oracle)."""
import numpy as np
import pytest
import torch

import sac_oracle as O
from sac_eager_torch import EagerSAC


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30))


@pytest.mark.parametrize("use_expert", [False, True])
def test_eager_update_equals_oracle(use_expert):
    cfg = O.Config(S=5, A=3, hidden=(32, 32), act="relu", B=16, model_hidden=(24, 24), epsilon=0.1)
    st = O.init_state(cfg, seed=3, with_models=use_expert, bias_scale=0.05, actor_gain=0.5, model_gain=0.3)
    eng = EagerSAC(st, cfg, use_expert=use_expert)
    st = st.astype(np.float64)
    nrm = O.Normalizers.identity(5, 3)
    rs = np.random.RandomState(0)
    N = 200
    buf = dict(s=rs.normal(size=(N, 5)).astype(np.float32), a=rs.uniform(-1, 1, (N, 3)).astype(np.float32),
               sp=rs.normal(size=(N, 5)).astype(np.float32), r=rs.normal(size=N).astype(np.float32),
               d=(rs.uniform(size=N) < 0.1).astype(np.float64))
    ex_s, ex_sp = rs.normal(size=(20, 5)).astype(np.float32), rs.normal(size=(20, 5)).astype(np.float32)
    t = lambda x: torch.tensor(np.asarray(x, np.float32))
    for _ in range(2):
        R = O.draw_step_randoms(rs, N, 16, 3, n_expert=20 if use_expert else 0,
                                gen=np.random.default_rng(1) if use_expert else None)
        b = O.gather(buf, R["idx"])
        ex = exo = None
        if use_expert:
            h1, h2 = R["sections"]
            ex = ((t(ex_s[h1]), t(ex_sp[h1]), t(O.f32_noise(R["noise_e1"]))),
                  (t(ex_s[h2]), t(ex_sp[h2]), t(O.f32_noise(R["noise_e2"]))), cfg.epsilon)
            exo = O.Expert(ex_s[h1], ex_sp[h1], ex_s[h2], ex_sp[h2], O.f32_noise(R["noise_e1"]),
                           O.f32_noise(R["noise_e2"]), cfg.epsilon)
        got = eng.update(*(t(x) for x in b), t(O.f32_noise(R["noise_t"])), t(O.f32_noise(R["noise_pi"])),
                         t(O.f32_noise(R["noise_alpha"])), ex)
        ref = O.sac_update(st, cfg, nrm, b, O.f32_noise(R["noise_t"]), O.f32_noise(R["noise_pi"]),
                           O.f32_noise(R["noise_alpha"]), expert=exo)
        for g, k in zip(got, ("q1_loss", "q2_loss", "p_loss", "alpha_loss")):
            assert abs(g - ref[k]) <= 1e-4 * abs(ref[k]) + 1e-6, (k, g, ref[k])
    for mine, theirs in [(eng.actor, st.actor), (eng.q[0], st.q[0]), (eng.q[1], st.q[1]),
                         (eng.qt[0], st.q_targ[0])]:
        for a, b in zip(mine, theirs):
            assert _rel(a.detach().numpy(), b) < 1e-4
    assert abs(float(eng.alpha) - float(st.alpha)) < 1e-6
    if use_expert:
        batches = [(buf["s"][:30], buf["a"][:30], buf["sp"][:30], buf["r"][:30]),
                   (buf["s"][30:60], buf["a"][30:60], buf["sp"][30:60], buf["r"][30:60])]
        lt = eng.model_fit_step([tuple(t(x) for x in bb) for bb in batches])
        lo = O.model_fit_step(st, cfg, nrm, batches)
        assert abs(lt - lo) <= 1e-5 * abs(lo)
        for a, b in zip(eng.models[1], st.models[1]):
            assert _rel(a.detach().numpy(), b) < 1e-4
