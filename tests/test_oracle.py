"""Pins the CPU oracle (test infrastructure) before it is trusted.

* the C MT19937 restatement vs NumPy's legacy RandomState (the reference's
  RNG, sac_eo/common/buffers.py:136, continuous_actors.py:351) and vs the
  committed golden vectors (tests/golden/rng_golden.npz);
* the closed-form backward of sac_oracle vs torch autograd (fp64) on the same
  forward formulas (reference: tf.GradientTape in SAC_expert.py:238-347);
* fp32 emulation vs fp64 reference over a short trajectory.
"""
import os

import numpy as np
import pytest

import sac_oracle as O
from mt_oracle import MTOracle

GOLD = os.path.join(os.path.dirname(__file__), "golden")


# ----------------------------------------------------------------- RNG
@pytest.mark.parametrize("seed", [0, 2773201285, 2590541744])
def test_mt_oracle_matches_numpy(seed):
    rs = np.random.RandomState(seed)
    mo = MTOracle(seed)
    for high in [1, 2, 3, 777, 5000, 2 ** 20, 10 ** 6, 4 * 10 ** 6, 2 ** 31]:
        assert np.array_equal(rs.randint(high, size=301), mo.randint(high, 301))
        assert np.array_equal(rs.normal(size=(7, 3)), mo.normal((7, 3)))   # odd: exercises the cache
    a, b = rs.get_state(), mo.get_state()
    assert np.array_equal(a[1], b[1]) and a[2] == b[2] and a[3] == b[3] and a[4] == b[4]


def test_mt_oracle_set_state_roundtrip():
    rs = np.random.RandomState(7)
    rs.normal(size=3)          # leaves a cached gaussian
    mo = MTOracle()
    mo.set_state(rs.get_state())
    assert np.array_equal(rs.normal(size=11), mo.normal(11))
    assert np.array_equal(rs.randint(999_999, size=64), mo.randint(999_999, 64))


def test_rng_golden_vectors():
    g = np.load(os.path.join(GOLD, "rng_golden.npz"))
    for key in [k for k in g.files if k.startswith("seed_") and k.endswith("_normal")]:
        name = key[: -len("_normal")]
        seed = int(name.split("_")[1])
        for high in g["highs"]:
            assert np.array_equal(MTOracle(seed).randint(int(high), 256), g[f"{name}_int_{int(high)}"])
        assert np.array_equal(MTOracle(seed).normal((256, 6)), g[f"{name}_normal"])
    mo = MTOracle(2590541744)
    assert np.array_equal(mo.randint(10 ** 6, 256), g["step_idx"])
    for k in ("noise_t", "noise_pi", "noise_alpha"):
        assert np.array_equal(mo.normal((256, 6)), g["step_" + k])


def test_seed_derivation_known_answer():
    """sac_eo/train.py:118-128 with --seed 0 (values recorded in the reference's
    sac_eo/logs/TEMPLOG_0 param.setup_kwargs)."""
    seeds = np.random.SeedSequence(0).generate_state(5)
    got = [int(np.random.SeedSequence(seeds[k]).generate_state(1)[0]) for k in range(5)]
    assert got[:4] == [2773201285, 397334063, 3968933684, 2590541744]
    assert got[4] == 3892593679


# ----------------------------------------------------------------- backward vs autograd
torch = pytest.importorskip("torch")


def _t(x):
    return torch.tensor(np.asarray(x, np.float64), dtype=torch.float64)


def _mlp(params, x, act):
    h = x
    n = len(params) // 2
    hs = []
    for l in range(n):
        z = h @ params[2 * l] + params[2 * l + 1]
        if l < n - 1:
            h = {"relu": torch.relu, "tanh": torch.tanh,
                 "elu": torch.nn.functional.elu}[act](z)
            hs.append(h)
        else:
            h = z
    return h


def _head_eval(mu, lraw, u):
    l = torch.clamp(lraw, -5.0, 2.0)
    std = torch.exp(l)
    x = mu + std * u
    z = (x - mu) / torch.exp(l)
    nlp = 0.5 * (z * z + 2 * l + np.log(2 * np.pi)).sum(-1)
    nlp = nlp + (2.0 * (np.log(2.0) - x - torch.nn.functional.softplus(-2.0 * x))).sum(-1)
    return torch.tanh(x), nlp


def _make(cfg, seed=3, bias_scale=0.1):
    st = O.init_state(cfg, seed=seed, with_models=True, bias_scale=bias_scale,
                      actor_gain=0.5, model_gain=0.3).astype(np.float64)
    rs = np.random.RandomState(seed + 10)
    B, S, A = cfg.B, cfg.S, cfg.A
    batch = (rs.normal(size=(B, S)), rs.uniform(-1, 1, (B, A)), rs.normal(size=(B, S)),
             rs.normal(size=B), (rs.uniform(size=B) < 0.2).astype(np.float64))
    noises = [rs.normal(size=(B, A)) for _ in range(3)]
    nrm = O.Normalizers(rs.normal(size=S) * 0.1, rs.uniform(0.5, 2, S), rs.normal(size=A) * 0.1,
                        rs.uniform(0.5, 2, A), rs.normal(size=S) * 0.1, rs.uniform(0.5, 2, S),
                        0.0, 1.0, 1.0).cast(np.float64)
    ne = 6
    ex = O.Expert(rs.normal(size=(ne // 2, S)), rs.normal(size=(ne // 2, S)),
                  rs.normal(size=(ne // 2, S)), rs.normal(size=(ne // 2, S)),
                  rs.normal(size=(ne // 2, A)), rs.normal(size=(ne // 2, A)), 0.3)
    return st, batch, noises, nrm, ex


@pytest.mark.parametrize("act", ["relu", "tanh", "elu"])
@pytest.mark.parametrize("use_expert", [False, True])
def test_oracle_backward_matches_autograd(act, use_expert):
    cfg = O.Config(S=5, A=3, hidden=(16, 12), act=act, B=32, model_hidden=(20, 18))
    st0, batch, noises, nrm, ex = _make(cfg)
    st1 = st0.copy()
    keep = {}
    O.sac_update(st1, cfg, nrm, batch, *noises, expert=ex if use_expert else None, keep=keep)
    s, a, sp, r, d = [_t(x) for x in batch]
    S = cfg.S
    nm = lambda x, m, dd: (x - _t(m)) / _t(dd)

    # critic grads (pre-Adam) vs autograd; target y from the oracle's own value
    y = _t(keep["y"])
    for k in range(2):
        P = [_t(w).requires_grad_() for w in st0.q[k]]
        q = _mlp(P, torch.cat([nm(s, nrm.s_mean, nrm.s_den), nm(a, nrm.a_mean, nrm.a_den)], 1), act)
        loss = torch.mean(0.5 * ((q - y[:, None]) ** 2).sum(-1))
        g = torch.autograd.grad(loss, P)
        for gg, mine in zip(g, keep["q%d_grads" % k]):
            np.testing.assert_allclose(mine, gg.numpy(), rtol=1e-9, atol=1e-12)

    # actor grads with the UPDATED critics and the PRE-update actor/alpha
    PA = [_t(w).requires_grad_() for w in st0.actor]
    LS = _t(st0.logstd).requires_grad_()
    Q = [[_t(w) for w in net] for net in st1.q]
    s_n = nm(s, nrm.s_mean, nrm.s_den)
    mu = _mlp(PA, s_n, act)
    pi, nlp = _head_eval(mu, LS.expand_as(mu), _t(noises[1]))
    xq = torch.cat([s_n, nm(pi, nrm.a_mean, nrm.a_den)], 1)
    minq = torch.minimum(_mlp(Q[0], xq, act), _mlp(Q[1], xq, act))
    alpha = float(st0.alpha)
    p = torch.mean(-alpha * nlp[:, None] - minq)
    if use_expert:
        M = [[_t(w) for w in net] for net in st0.models]
        sq = []
        for k, (se, spe, ne) in enumerate([(ex.s1, ex.sp1, ex.noise1), (ex.s2, ex.sp2, ex.noise2)]):
            se_n = nm(_t(se), nrm.s_mean, nrm.s_den)
            mue = _mlp(PA, se_n, act)
            ca = torch.tanh(mue + torch.exp(torch.clamp(LS, -5, 2)) * _t(ne))
            om = _mlp(M[k], torch.cat([se_n, nm(ca, nrm.a_mean, nrm.a_den)], 1), cfg.model_act)
            sp_hat = _t(se) + (om[:, :S] * _t(nrm.d_den) + _t(nrm.d_mean))
            sq.append(((_t(spe) - sp_hat) ** 2).sum(-1))
        mse = torch.mean(0.5 * (sq[0] + sq[1]))
        p = (1 - ex.epsilon) * p + ex.epsilon * mse
    g = torch.autograd.grad(p, PA + [LS])
    for gg, mine in zip(g[:-1], keep["actor_grads"]):
        np.testing.assert_allclose(mine, gg.numpy(), rtol=1e-7, atol=1e-10)
    np.testing.assert_allclose(keep["g_logstd"], g[-1].numpy(), rtol=1e-7, atol=1e-10)

    # alpha grad: d(-alpha*mean(-nlp + H))/dalpha with the UPDATED actor
    mu3 = _mlp([_t(w) for w in st1.actor], s_n, act)
    _, nlp3 = _head_eval(mu3, _t(st1.logstd).expand_as(mu3), _t(noises[2]))
    al = torch.tensor(alpha, dtype=torch.float64, requires_grad=True)
    (ga,) = torch.autograd.grad(-al * torch.mean(-nlp3 + cfg.target_entropy), al)
    np.testing.assert_allclose(float(keep["g_alpha"]), ga.item(), rtol=1e-10)


def test_min_tie_split():
    """TF _MinOrMaxGrad splits the gradient of reduce_min equally on ties."""
    cfg = O.Config(S=3, A=1, hidden=(8, 8), B=8)
    st = O.init_state(cfg, seed=2).astype(np.float64)
    st.q[1] = [w.copy() for w in st.q[0]]          # identical critics -> every row ties
    st.opt_q[1] = O.AdamState.zeros_like(st.q[1])
    rs = np.random.RandomState(0)
    batch = (rs.normal(size=(8, 3)), rs.uniform(-1, 1, (8, 1)), rs.normal(size=(8, 3)),
             rs.normal(size=8), np.zeros(8))
    keep = {}
    O.sac_update(st, cfg, O.Normalizers.identity(3, 1).cast(np.float64), batch,
                 *[rs.normal(size=(8, 1)) for _ in range(3)], keep=keep)
    assert np.array_equal(keep["q1p"], keep["q2p"])


def test_fp32_emulation_tracks_fp64():
    cfg = O.Config(S=17, A=6, B=64)
    st64 = O.init_state(cfg, seed=1).astype(np.float64)
    st32 = O.init_state(cfg, seed=1)
    rs = np.random.RandomState(0)
    N = 500
    buf = dict(s=rs.normal(size=(N, 17)).astype(np.float32), a=rs.uniform(-1, 1, (N, 6)).astype(np.float32),
               sp=rs.normal(size=(N, 17)).astype(np.float32), r=rs.normal(size=N).astype(np.float32),
               d=np.zeros(N))
    nrm = O.Normalizers.identity(17, 6)
    g64, g32 = np.random.RandomState(3), np.random.RandomState(3)
    for _ in range(30):
        R1 = O.draw_step_randoms(g64, N, 64, 6)
        R2 = O.draw_step_randoms(g32, N, 64, 6)
        n = [O.f32_noise(R1[k]) for k in ("noise_t", "noise_pi", "noise_alpha")]
        s64 = O.sac_update(st64, cfg, nrm, O.gather(buf, R1["idx"]), *n)
        s32 = O.sac_update(st32, cfg, nrm, O.gather(buf, R2["idx"]), *n)
        for k in ("q1_loss", "q2_loss"):
            assert abs(s64[k] - s32[k]) <= 1e-4 * abs(s64[k]) + 1e-7


def test_model_fit_step_matches_autograd():
    cfg = O.Config(S=4, A=2, hidden=(8, 8), B=16, model_hidden=(10, 12))
    st = O.init_state(cfg, seed=5, with_models=True, bias_scale=0.1, model_gain=0.5).astype(np.float64)
    rs = np.random.RandomState(1)
    nrm = O.Normalizers(rs.normal(size=4) * .1, rs.uniform(.5, 2, 4), rs.normal(size=2) * .1,
                        rs.uniform(.5, 2, 2), rs.normal(size=4) * .1, rs.uniform(.5, 2, 4), 0.2, 1.5, 1.0)
    batches = [(rs.normal(size=(9, 4)), rs.uniform(-1, 1, (9, 2)), rs.normal(size=(9, 4)),
                rs.normal(size=9)) for _ in range(2)]
    M = [[_t(w).requires_grad_() for w in net] for net in st.models]
    tot = 0
    for k, (s, a, sp, r) in enumerate(batches):
        x = torch.cat([(_t(s) - _t(nrm.s_mean)) / _t(nrm.s_den), (_t(a) - _t(nrm.a_mean)) / _t(nrm.a_den)], 1)
        out = _mlp(M[k], x, "relu")
        dn = ((_t(sp) - _t(s)) - _t(nrm.d_mean)) / _t(nrm.d_den)
        rn = (_t(r) - nrm.r_mean) / nrm.r_den
        tot = tot + torch.mean(0.5 * ((dn - out[:, :4]) ** 2).sum(-1) + 0.5 * (rn - out[:, 4]) ** 2)
    g = torch.autograd.grad(tot, M[0] + M[1])
    # reproduce the oracle's first Adam step from the autograd gradients
    ref = st.copy()
    O.adam_step(ref.models[0] + ref.models[1], [x.numpy() for x in g], ref.opt_model, cfg.lr_model, np.float64)
    loss = O.model_fit_step(st, cfg, nrm, batches)
    assert abs(loss - tot.item()) < 1e-12
    for w1, w2 in zip(st.models[0] + st.models[1], ref.models[0] + ref.models[1]):
        np.testing.assert_allclose(w1, w2, rtol=1e-12, atol=1e-14)


def test_rollout_oracle_consumes_one_draw_per_step():
    """oracle.rollout (samplers.py:73-122): one normal(size=(n, A)) per step, s_{t+1} = sp_t,
    d all False; deterministic draws nothing."""
    cfg = O.Config(S=3, A=2, hidden=(8, 8), act="tanh", B=4, model_hidden=(8, 8))
    st = O.init_state(cfg, seed=3, with_models=True).astype(np.float64)
    nrm = O.Normalizers.identity(3, 2)
    s0 = np.random.RandomState(1).normal(size=(5, 3))
    rs = np.random.RandomState(7)
    s, a, r, sp, d = O.rollout(st, cfg, nrm, s0, 4, 0, rs)
    ref = np.random.RandomState(7)
    for _ in range(4):
        ref.normal(size=(5, 2))
    assert rs.get_state()[2] == ref.get_state()[2] and np.array_equal(rs.get_state()[1], ref.get_state()[1])
    assert s.shape == (5, 4, 3) and a.shape == (5, 4, 2) and r.shape == (5, 4) and d.shape == (5, 4)
    assert np.array_equal(s[:, 1:], sp[:, :-1]) and not d.any()
    assert np.all(np.abs(a) <= 1.0)
    rs2 = np.random.RandomState(7)
    O.rollout(st, cfg, nrm, s0, 4, 0, rs2, deterministic=True)
    assert rs2.get_state()[2] == np.random.RandomState(7).get_state()[2]


def test_mt_unrolled_recurrence():
    """The device sampler's word recurrence (csrc/k_sac.hip rng_twist): MT19937's raw words
    satisfy x[n] = x[n-227] ^ g(n-624) and, unrolled, x[n] = x[n-681] ^ g(n-624) ^ g(n-851) ^
    g(n-1078) with g(m) = twist(x[m], x[m+1]).  Raw blocks come from NumPy's own state after
    every 624 full-range draws."""
    rs = np.random.RandomState(2773201285)
    blocks = []
    for _ in range(6):
        rs.randint(0, 2 ** 32, size=624, dtype=np.uint64)   # warm: position at a block edge
        blocks.append(np.array(rs.get_state()[1], dtype=np.uint64))
    x = np.concatenate(blocks)

    def g(m):
        y = (x[m] & 0x80000000) | (x[m + 1] & 0x7FFFFFFF)
        return (y >> 1) ^ np.where(y & 1, 0x9908B0DF, 0).astype(np.uint64)

    n = np.arange(624, len(x))
    assert np.array_equal(x[n], x[n - 227] ^ g(n - 624))
    n = np.arange(1078, len(x))
    assert np.array_equal(x[n], x[n - 681] ^ g(n - 624) ^ g(n - 851) ^ g(n - 1078))


@pytest.mark.parametrize("act", ["relu", "tanh"])
def test_oracle_one_model_expert_matches_autograd(act):
    """--num_models 1 (SAC_expert.py:273-296): every expert row, in order, through model 0;
    MSE = mean over the rows of 0.5 ||sp_e - sp_pred||^2."""
    cfg = O.Config(S=5, A=3, hidden=(16, 12), act=act, B=32, model_hidden=(20, 18))
    st0, batch, noises, nrm, _ = _make(cfg, seed=4)
    rs = np.random.RandomState(21)
    ne = 7                                     # odd: one model needs no equal halves
    ex = O.Expert(rs.normal(size=(ne, 5)), rs.normal(size=(ne, 5)), None, None, rs.normal(size=(ne, 3)), None, 0.4)
    st1 = st0.copy()
    keep = {}
    stats = O.sac_update(st1, cfg, nrm, batch, *noises, expert=ex, keep=keep)
    s = _t(batch[0])
    nm = lambda x, m, dd: (x - _t(m)) / _t(dd)
    PA = [_t(w).requires_grad_() for w in st0.actor]
    LS = _t(st0.logstd).requires_grad_()
    Q = [[_t(w) for w in net] for net in st1.q]
    s_n = nm(s, nrm.s_mean, nrm.s_den)
    mu = _mlp(PA, s_n, act)
    pi, nlp = _head_eval(mu, LS.expand_as(mu), _t(noises[1]))
    xq = torch.cat([s_n, nm(pi, nrm.a_mean, nrm.a_den)], 1)
    minq = torch.minimum(_mlp(Q[0], xq, act), _mlp(Q[1], xq, act))
    p = torch.mean(-float(st0.alpha) * nlp[:, None] - minq)
    se_n = nm(_t(ex.s1), nrm.s_mean, nrm.s_den)
    ca = torch.tanh(_mlp(PA, se_n, act) + torch.exp(torch.clamp(LS, -5, 2)) * _t(ex.noise1))
    om = _mlp([_t(w) for w in st0.models[0]], torch.cat([se_n, nm(ca, nrm.a_mean, nrm.a_den)], 1), cfg.model_act)
    sp_hat = _t(ex.s1) + (om[:, :5] * _t(nrm.d_den) + _t(nrm.d_mean))
    mse = torch.mean(0.5 * ((_t(ex.sp1) - sp_hat) ** 2).sum(-1))
    p = (1 - ex.epsilon) * p + ex.epsilon * mse
    assert abs(stats["mse_loss"] - mse.item()) < 1e-10 and abs(stats["p_loss"] - p.item()) < 1e-10
    g = torch.autograd.grad(p, PA + [LS])
    for gg, mine in zip(g[:-1], keep["actor_grads"]):
        np.testing.assert_allclose(mine, gg.numpy(), rtol=1e-7, atol=1e-10)
    np.testing.assert_allclose(keep["g_logstd"], g[-1].numpy(), rtol=1e-7, atol=1e-10)


@pytest.mark.parametrize("nmodels,max_norm,dclip,rclip", [(2, 0.05, 0.0, 0.0), (1, 0.02, 0.3, 0.5),
                                                          (2, 100.0, 0.0, 0.0)])
def test_model_fit_clips_and_global_norm(nmodels, max_norm, dclip, rclip):
    """--model_max_grad_norm (mbrl_onpolicy_alg.py:315-317: clip_by_global_norm to
    max_norm * num_models) and the get_loss target clips (continuous_models.py:284-296),
    against autograd + TF's clip_by_global_norm formula; a large max_norm leaves the step
    unchanged."""
    cfg = O.Config(S=4, A=2, hidden=(8, 8), B=16, model_hidden=(10, 12))
    st = O.init_state(cfg, seed=6, with_models=True, bias_scale=0.1, model_gain=0.5).astype(np.float64)
    rs = np.random.RandomState(2)
    nrm = O.Normalizers(rs.normal(size=4) * .1, rs.uniform(.5, 2, 4), rs.normal(size=2) * .1,
                        rs.uniform(.5, 2, 2), rs.normal(size=4) * .1, rs.uniform(.5, 2, 4), 0.2, 1.5, 1.0)
    batches = [(rs.normal(size=(9, 4)), rs.uniform(-1, 1, (9, 2)), rs.normal(size=(9, 4)) * 3,
                rs.normal(size=9) * 3) for _ in range(nmodels)]
    M = [[_t(w).requires_grad_() for w in net] for net in st.models[:nmodels]]
    tot = 0
    for k, (s, a, sp, r) in enumerate(batches):
        x = torch.cat([(_t(s) - _t(nrm.s_mean)) / _t(nrm.s_den), (_t(a) - _t(nrm.a_mean)) / _t(nrm.a_den)], 1)
        out = _mlp(M[k], x, "relu")
        dn = ((_t(sp) - _t(s)) - _t(nrm.d_mean)) / _t(nrm.d_den)
        rn = (_t(r) - nrm.r_mean) / nrm.r_den
        if dclip:
            dn = torch.clamp(dn, -dclip, dclip)
        if rclip:
            rn = torch.clamp(rn, -rclip, rclip)
        tot = tot + torch.mean(0.5 * ((dn - out[:, :4]) ** 2).sum(-1) + 0.5 * (rn - out[:, 4]) ** 2)
    flat = [w for net in M for w in net]
    g = [x.numpy() for x in torch.autograd.grad(tot, flat)]
    clip = max_norm * nmodels
    norm = np.sqrt(sum(np.sum(x * x) for x in g))
    g = [x * (clip * min(1.0 / norm, 1.0 / clip)) for x in g]
    ref = st.copy()
    O.adam_step([w for k in range(nmodels) for w in ref.models[k]], g, ref.opt_model, cfg.lr_model, np.float64)
    loss = O.model_fit_step(st, cfg, nrm, batches, max_grad_norm=max_norm, delta_clip_loss=dclip,
                            reward_clip_loss=rclip)
    assert abs(loss - tot.item()) < 1e-12
    for k in range(nmodels):
        for w1, w2 in zip(st.models[k], ref.models[k]):
            np.testing.assert_allclose(w1, w2, rtol=1e-12, atol=1e-14)
    if nmodels == 1:                            # model 1 untouched
        assert st.opt_model.t == 1


@pytest.mark.parametrize("gauss,sep,scale,max_norm,dclip", [
    (True, False, False, None, 0.0), (True, False, True, None, 0.4), (False, True, False, None, 0.0),
    (True, True, True, 0.05, 0.0), (True, True, False, None, 0.3)])
def test_model_fit_gaussian_and_reward_net_match_autograd(gauss, sep, scale, max_norm, dclip):
    """GaussianModel.get_loss (continuous_models.py:101-131: the NLL with the trainable logstd,
    --scale_model_loss as a stop-gradient factor) and --separate_reward_nn (base_world_model.py:32-37,
    :72-74: the model net predicts the S deltas, the reward net the reward) against autograd, with
    one Adam over model.trainable (nn, logstd, reward nn per model) and the global-norm clip."""
    cfg = O.Config(S=4, A=2, hidden=(8, 8), B=16, model_hidden=(10, 12), gaussian_model=gauss,
                   separate_reward_nn=sep, scale_model_loss=scale, reward_hidden=(7, 9), reward_act="tanh",
                   reward_loss_coef=0.7)
    st = O.init_state(cfg, seed=8, with_models=True, bias_scale=0.1, model_gain=0.5, model_std_mult=0.8,
                      reward_gain=0.4).astype(np.float64)
    rs = np.random.RandomState(3)
    nrm = O.Normalizers(rs.normal(size=4) * .1, rs.uniform(.5, 2, 4), rs.normal(size=2) * .1,
                        rs.uniform(.5, 2, 2), rs.normal(size=4) * .1, rs.uniform(.5, 2, 4), 0.2, 1.5, 1.0)
    batches = [(rs.normal(size=(9, 4)), rs.uniform(-1, 1, (9, 2)), rs.normal(size=(9, 4)) * 2,
                rs.normal(size=9) * 2) for _ in range(2)]
    V = [[_t(w).requires_grad_() for w in st.model_vars(k)] for k in range(2)]
    tot = 0
    for k, (s, a, sp, r) in enumerate(batches):
        x = torch.cat([(_t(s) - _t(nrm.s_mean)) / _t(nrm.s_den), (_t(a) - _t(nrm.a_mean)) / _t(nrm.a_den)], 1)
        nn = V[k][:6]
        out = _mlp(nn, x, "relu")
        rp = _mlp(V[k][-6:], x, "tanh")[:, 0] if sep else out[:, 4]
        dn = ((_t(sp) - _t(s)) - _t(nrm.d_mean)) / _t(nrm.d_den)
        if dclip:
            dn = torch.clamp(dn, -dclip, dclip)
        rn = (_t(r) - nrm.r_mean) / nrm.r_den
        if gauss:
            l = V[k][6]
            q = (dn - out[:, :4]) / torch.exp(l)
            sc = torch.mean(torch.exp(l) ** 2).detach() if scale else 1.0
            dl = sc * 0.5 * (q * q + 2 * l + float(np.log(np.float32(2 * np.pi)))).sum(-1)   # TF: a float32 constant
        else:
            dl = 0.5 * ((dn - out[:, :4]) ** 2).sum(-1)
        tot = tot + torch.mean(dl + 0.7 * 0.5 * (rn - rp) ** 2)
        if k == 0:
            assert abs(O.model_loss(st, cfg, nrm, 0, s, sp, a, r, delta_clip_loss=dclip)
                       - torch.mean(dl + 0.7 * 0.5 * (rn - rp) ** 2).item()) < 1e-12
    flat = [w for vs in V for w in vs]
    g = [x.numpy() for x in torch.autograd.grad(tot, flat)]
    if max_norm:
        clip = max_norm * 2
        norm = np.sqrt(sum(np.sum(x * x) for x in g))
        g = [x * (clip * min(1.0 / norm, 1.0 / clip)) for x in g]
    ref = st.copy()
    O.adam_step(ref.model_all_vars(), g, ref.opt_model, cfg.lr_model, np.float64)
    loss = O.model_fit_step(st, cfg, nrm, batches, max_grad_norm=max_norm, delta_clip_loss=dclip)
    assert abs(loss - tot.item()) < 1e-12
    for w1, w2 in zip(st.model_all_vars(), ref.model_all_vars()):
        np.testing.assert_allclose(w1, w2, rtol=1e-12, atol=1e-14)
    if gauss:                         # the logstd variables moved (they are trained)
        assert not np.array_equal(st.model_logstd[0], O.init_state(cfg, seed=8, with_models=True,
                                  model_std_mult=0.8).model_logstd[0])


def test_gaussian_model_noise_order():
    """GaussianModel draws normal(size=(n, S)) in sample(deterministic=False) and in every step
    (continuous_models.py:36-70): the rollout draws the actor's (n, A) then the model's (n, S) per
    step; _calc_disc the actor's, then model 0's, then model 1's (SAC_expert.py:442-446)."""
    cfg = O.Config(S=3, A=2, hidden=(8, 8), act="tanh", B=4, model_hidden=(8, 8), gaussian_model=True)
    st = O.init_state(cfg, seed=3, with_models=True).astype(np.float64)
    nrm = O.Normalizers.identity(3, 2)
    s0 = np.random.RandomState(1).normal(size=(5, 3))
    rs = np.random.RandomState(7)
    s, a, r, sp, d = O.rollout(st, cfg, nrm, s0, 2, 0, rs)
    ref = np.random.RandomState(7)
    for _ in range(2):
        ref.normal(size=(5, 2))
        ref.normal(size=(5, 3))
    assert rs.get_state()[2] == ref.get_state()[2] and np.array_equal(rs.get_state()[1], ref.get_state()[1])
    rs2 = np.random.RandomState(9)
    O.rollout(st, cfg, nrm, s0, 2, 0, rs2, deterministic=True)      # the model still draws
    ref2 = np.random.RandomState(9)
    ref2.normal(size=(5, 3))
    ref2.normal(size=(5, 3))
    assert rs2.get_state()[2] == ref2.get_state()[2]
    rs3 = np.random.RandomState(4)
    O.calc_disc(st, cfg, nrm, s0, None, rs=rs3)
    ref3 = np.random.RandomState(4)
    ref3.normal(size=(5, 2))
    ref3.normal(size=(5, 3))
    ref3.normal(size=(5, 3))
    assert rs3.get_state()[2] == ref3.get_state()[2]
    assert abs(O.model_entropy(st, cfg, 0) - 0.5 * np.sum(2 * st.model_logstd[0] + np.log(2 * np.pi) + 1)) < 1e-5


@pytest.mark.parametrize("use_expert", [False, True])
def test_oracle_layer_norm_actor_matches_autograd(use_expert):
    """--actor_layer_norm (nn_utils.py:110-119): Dense -> LayerNormalization(eps 1e-3) -> tanh
    on the actor's layer 0; the closed-form actor gradients (incl. gamma / beta) vs autograd."""
    cfg = O.Config(S=5, A=3, hidden=(16, 12), act="relu", B=32, model_hidden=(20, 18), layer_norm=True)
    st0 = O.init_state(cfg, seed=7, with_models=True, bias_scale=0.1, actor_gain=0.5,
                       model_gain=0.3).astype(np.float64)
    _, batch, noises, nrm, ex = _make(O.Config(S=5, A=3, hidden=(16, 12), act="relu", B=32, model_hidden=(20, 18)))
    st1 = st0.copy()
    keep = {}
    O.sac_update(st1, cfg, nrm, batch, *noises, expert=ex if use_expert else None, keep=keep)
    nm = lambda x, m, dd: (x - _t(m)) / _t(dd)

    def actor(P, x):
        z = x @ P[0] + P[1]
        mu = z.mean(-1, keepdim=True)
        var = ((z - mu) ** 2).mean(-1, keepdim=True)
        h = torch.tanh(P[2] * (z - mu) / torch.sqrt(var + 1e-3) + P[3])
        return _mlp(P[4:], h, "relu")
    PA = [_t(w).requires_grad_() for w in st0.actor]
    LS = _t(st0.logstd).requires_grad_()
    Q = [[_t(w) for w in net] for net in st1.q]
    s_n = nm(_t(batch[0]), nrm.s_mean, nrm.s_den)
    pi, nlp = _head_eval(actor(PA, s_n), LS.expand(32, 3), _t(noises[1]))
    xq = torch.cat([s_n, nm(pi, nrm.a_mean, nrm.a_den)], 1)
    p = torch.mean(-float(st0.alpha) * nlp[:, None] - torch.minimum(_mlp(Q[0], xq, "relu"), _mlp(Q[1], xq, "relu")))
    if use_expert:
        M = [[_t(w) for w in net] for net in st0.models]
        sq = []
        for k, (se, spe, ne) in enumerate([(ex.s1, ex.sp1, ex.noise1), (ex.s2, ex.sp2, ex.noise2)]):
            se_n = nm(_t(se), nrm.s_mean, nrm.s_den)
            ca = torch.tanh(actor(PA, se_n) + torch.exp(torch.clamp(LS, -5, 2)) * _t(ne))
            om = _mlp(M[k], torch.cat([se_n, nm(ca, nrm.a_mean, nrm.a_den)], 1), cfg.model_act)
            sq.append(((_t(spe) - (_t(se) + (om[:, :5] * _t(nrm.d_den) + _t(nrm.d_mean)))) ** 2).sum(-1))
        p = (1 - ex.epsilon) * p + ex.epsilon * torch.mean(0.5 * (sq[0] + sq[1]))
    g = torch.autograd.grad(p, PA + [LS])
    assert len(keep["actor_grads"]) == 8
    for gg, mine in zip(g[:-1], keep["actor_grads"]):
        np.testing.assert_allclose(mine, gg.numpy(), rtol=1e-7, atol=1e-10)
    np.testing.assert_allclose(keep["g_logstd"], g[-1].numpy(), rtol=1e-7, atol=1e-10)
