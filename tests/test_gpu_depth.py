"""Nets of any depth and more than two world models on the device, against the oracle (round 6).

The reference builds every net with ``create_nn`` over a ``layers`` list of any length
(sac_eo/common/nn_utils.py:100-138; ``--actor_layers`` / ``--critic_layers`` / ``--model_layers`` /
``--reward_layers`` are ``nargs='+'``, train_parser.py:56-57, :107-108) and fits ``--num_models``
world models in one Adam step (mbrl_onpolicy_alg.py:301-319), the SAC-EO expert term using the
first two of ``np.array_split(perm, num_models)`` (SAC_expert.py:297-336).  Nets of other than two
hidden layers run libsacx's generic plans (every Dense layer a problem of its level's forward /
dX / dW launch, the heads on the row kernels); ``SACX_GENERIC=1`` runs those plans at two layers,
which checks them against the same oracle the fused plans meet.

Compared (fp32 device vs fp64 oracle, the bars of test_gpu_engine.py): one update's four losses
(2e-5 relative) and every gradient through Adam's first moment (2e-4 relative to the tensor's max);
a 60-update graph-replayed trajectory (Q losses 1e-4, alpha loss 1e-3) with the device stream
bit-exact; graph == eager bit for bit; model-fit steps (losses 1e-4, weights 5e-5); the object
calls, the rollout and the diagnostics (2e-5 / 1e-4)."""
import numpy as np
import pytest

import sac_oracle as O
from helpers import B1, make_pair, oracle_step, relerr

pytestmark = pytest.mark.gpu


def _same_stream(eng, rs):
    dev, ref = eng.rng_get_state(), rs.get_state()
    return np.array_equal(dev[1], ref[1]) and dev[2] == ref[2] and dev[3] == ref[3] and dev[4] == ref[4]


def _adam_grads(eng, net, B):
    """The gradient of every Dense layer of `net` from Adam's first moment (m_1 = g (1 - beta_1))."""
    m = eng.v["adam_m"][0]
    out = []
    i = 0
    while f"{net}.l{i}" in eng.segments:
        seg = eng.segments[f"{net}.l{i}"]
        off = seg["offset"] // 4
        w = m[off: off + seg["rows"] * seg["cols"]].cpu().numpy().reshape(seg["rows"], seg["cols"]) / B1
        out += [w[:-1], w[-1]]
        i += 1
    return out


CASES = {
    # name: make_pair keyword arguments
    "actor3": dict(hidden=(96, 64, 80)),
    "actor1": dict(hidden=(112,)),
    "critic3": dict(hidden=(64, 64), wm=dict(critic_hidden=(80, 48, 32))),
    "critic1": dict(hidden=(64, 64), wm=dict(critic_hidden=(96,))),
    "all4": dict(hidden=(64, 48, 48, 32), wm=dict(critic_hidden=(64, 64, 32, 48)), act="tanh"),
    "ln3": dict(hidden=(64, 80, 48), layer_norm=True),
    "ln1": dict(hidden=(64,), layer_norm=True),
    "pss3": dict(hidden=(64, 64, 64), per_state_std=True, act="elu"),
    "generic2": dict(hidden=(96, 64), generic=True),
    "eo_models3": dict(hidden=(64, 64), use_expert=True, model_hidden=(96, 64, 80)),
    "eo_models1": dict(hidden=(64, 64, 64), use_expert=True, model_hidden=(128,)),
    "eo_nm3": dict(hidden=(64, 64), use_expert=True, model_hidden=(96, 96), num_models=3, ne=20),
    "eo_nm4_deep": dict(hidden=(48, 64, 48), use_expert=True, model_hidden=(64, 96, 64), num_models=4, ne=16,
                        wm=dict(critic_hidden=(64, 32, 64))),
    "eo_generic2": dict(hidden=(64, 64), use_expert=True, model_hidden=(96, 128), generic=True),
}


def _pair(monkeypatch, case, B=64, seed=0, **over):
    kw = dict(CASES[case])
    kw.update(over)
    if kw.pop("generic", False):
        monkeypatch.setenv("SACX_GENERIC", "1")
    kw.setdefault("ne", 12)
    kw.setdefault("act", "relu")
    out = make_pair(B=B, seed=seed, normalizers="random", **kw)
    monkeypatch.delenv("SACX_GENERIC", raising=False)
    return out


@pytest.mark.parametrize("case", list(CASES))
def test_one_update_any_depth(gpu_available, monkeypatch, case):
    B = 64
    eng, ocfg, st, buf, nrm, expert = _pair(monkeypatch, case, B=B, seed=3)
    eo = expert is not None
    nm = eng.cfg.num_models
    N = buf["r"].shape[0]
    rs = np.random.RandomState(17)
    gen = np.random.default_rng(4)
    eng.rng_set_state(rs.get_state())
    R = O.draw_step_randoms(rs, N, B, ocfg.A, n_expert=eng.cfg.expert_batch if eo else 0, gen=gen, n_models=nm)
    if eo and nm > 1:
        eng.push_perms(R["perm"][None])
    keep = {}
    ref = oracle_step(st, ocfg, nrm, buf, R, expert, keep)
    eng.step(1, eager=True)
    eng.sync()
    row = eng.stats(1)[0]
    for i, k in enumerate(("q1_loss", "q2_loss", "p_loss", "alpha_loss")):
        assert abs(row[i] - ref[k]) <= 2e-5 * abs(ref[k]) + 1e-7, (k, row[i], ref[k])
    if eo:
        assert abs(row[5] - ref["mse_loss"]) <= 2e-5 * abs(ref["mse_loss"]), (row[5], ref["mse_loss"])
    assert np.array_equal(eng.v["slot0.idx"][0].cpu().numpy(), R["idx"])
    assert _same_stream(eng, rs)
    for k in range(2):
        for gd, go in zip(_adam_grads(eng, f"q{k}", B), keep[f"q{k}_grads"]):
            assert relerr(gd, go) < 2e-4, (f"q{k}", relerr(gd, go))
        for a_, b_ in zip(eng.get_net(f"t{k}"), st.q_targ[k]):        # Polyak
            assert np.max(np.abs(a_ - b_)) < 1e-5
    ga = _adam_grads(eng, "actor", B)
    go = list(keep["actor_grads"])
    if ocfg.layer_norm:               # the oracle's list carries gamma / beta after b0; compare the Dense layers
        go = go[:2] + go[4:]
    assert len(ga) == len(go)
    for i, (gd, gr) in enumerate(zip(ga, go)):
        assert relerr(gd, gr) < 2e-4, ("actor", i, relerr(gd, gr))
    eng.close()


@pytest.mark.parametrize("case", ["all4", "eo_nm4_deep", "ln1", "generic2"])
def test_trajectory_any_depth(gpu_available, monkeypatch, case):
    """60 graph-replayed updates (graphs of 8 with the sampler forked ahead, alpha branches folded
    into the next update) against 60 oracle updates; the device stream bit-exact at the end."""
    B = 128
    eng, ocfg, st, buf, nrm, expert = _pair(monkeypatch, case, B=B, seed=11)
    eo = expert is not None
    nm = eng.cfg.num_models
    N = buf["r"].shape[0]
    rs = np.random.RandomState(123)
    gen = np.random.default_rng(77)
    eng.rng_set_state(rs.get_state())
    steps = 60
    Rs = [O.draw_step_randoms(rs, N, B, ocfg.A, n_expert=eng.cfg.expert_batch if eo else 0, gen=gen, n_models=nm)
          for _ in range(steps)]
    if eo:
        eng.push_perms(np.stack([R["perm"] for R in Rs]))
    eng.step(steps)
    eng.sync()
    dev = eng.stats(steps)
    ref = np.array([[o["q1_loss"], o["q2_loss"], o["alpha_loss"]]
                    for o in (oracle_step(st, ocfg, nrm, buf, R, expert) for R in Rs)])
    rel = np.abs(dev[:, :2] - ref[:, :2]) / np.abs(ref[:, :2])
    assert rel.max() < 1e-4, rel.max()
    rel_a = np.abs(dev[:, 3] - ref[:, 2]) / np.abs(ref[:, 2])
    assert rel_a.max() < 1e-3, rel_a.max()
    assert _same_stream(eng, rs)
    eng.close()


@pytest.mark.parametrize("case", ["actor3", "eo_nm3", "critic1"])
def test_graph_equals_eager_any_depth(gpu_available, monkeypatch, case):
    """The generic plan replayed from graphs == the same launches eager, bit for bit (19 updates)."""
    outs = []
    n = 19
    for eager in (True, False):
        eng, ocfg, st, buf, nrm, _ = _pair(monkeypatch, case, B=64, seed=21)
        eng.rng_set_state(np.random.RandomState(5).get_state())
        if eng.cfg.use_expert:
            rs = np.random.RandomState(8)
            eng.push_perms(np.stack([rs.permutation(eng.cfg.expert_batch) for _ in range(n)]))
        eng.step(n, eager=eager)
        eng.sync()
        outs.append((eng.stats(n).copy(), eng.v["params"].cpu().numpy().copy()))
        eng.close()
    assert np.array_equal(outs[0][0], outs[1][0])
    assert np.array_equal(outs[0][1], outs[1][1])


FIT = {
    "deep3": dict(model_hidden=(96, 64, 80)),
    "one": dict(model_hidden=(128,)),
    "nm3": dict(model_hidden=(96, 96), num_models=3),
    "nm5_clip": dict(model_hidden=(64, 96), num_models=5, model_max_grad_norm=0.05),
    "gauss_reward_deep": dict(model_hidden=(64, 48, 64), num_models=3,
                              wm=dict(gaussian_model=True, scale_model_loss=True, separate_reward_nn=True,
                                      reward_hidden=(48, 32, 40), reward_act="tanh")),
    "reward_mixed_depth": dict(model_hidden=(64,), wm=dict(separate_reward_nn=True, reward_hidden=(32, 48, 40),
                                                           reward_act="elu")),
}


@pytest.mark.parametrize("case", list(FIT))
def test_model_fit_any_depth(gpu_available, case):
    """sacx_model_fit of nm models of any depth (and reward nets of another depth): 2 eager steps, 3
    graph-replayed ones, the summed loss of each step and every model variable against the oracle."""
    kw = dict(FIT[case])
    nm = kw.get("num_models", 2)
    max_norm = kw.get("model_max_grad_norm", 0.0)
    eng, ocfg, st, buf, nrm, _ = make_pair(act="relu", hidden=(64, 64), B=64, seed=33, use_expert=True,
                                           normalizers="random", ne=12, **kw)
    N = buf["r"].shape[0]
    mb = eng.cfg.model_batch
    idx = np.random.RandomState(13).randint(N, size=(5, nm, mb))
    eng.model_fit(idx[:2], eager=True)
    eng.model_fit(idx[2:], eager=False)
    eng.sync()
    dev = eng.model_stats(5)
    ref = []
    for j in range(5):
        batches = [(buf["s"][idx[j, k]], buf["a"][idx[j, k]], buf["sp"][idx[j, k]], buf["r"][idx[j, k]])
                   for k in range(nm)]
        ref.append(O.model_fit_step(st, ocfg, nrm, batches, max_grad_norm=max_norm or None))
    ref = np.array(ref)
    assert np.max(np.abs(dev - ref) / np.abs(ref)) < 1e-4, (dev, ref)
    for k in range(nm):
        for a_, b_ in zip(eng.get_net(f"m{k}"), st.models[k]):
            assert np.max(np.abs(a_ - b_)) < 5e-5
        if ocfg.gaussian_model:
            assert np.max(np.abs(eng.get_model_logstd(k) - st.model_logstd[k])) < 5e-5
        if ocfg.separate_reward_nn:
            for a_, b_ in zip(eng.get_net(f"r{k}"), st.reward_nets[k]):
                assert np.max(np.abs(a_ - b_)) < 5e-5
    assert eng.ctl()["t_model"] == 5
    eng.close()


def _rows(n, S, A, seed=0):
    r = np.random.RandomState(seed)
    s = (r.normal(size=(n, S)) * 1.5).astype(np.float32)
    a = r.uniform(-1, 1, (n, A)).astype(np.float32)
    sp = (s + r.normal(size=(n, S)) * 0.2).astype(np.float32)
    return s, a, sp


def test_objects_any_depth(gpu_available):
    """actor.evaluate / sample, QCritic._forward / value and MSEModel.sample of nets with 3 / 1 / 4
    hidden layers: within 2e-5 of the oracle, the device stream bit-exact."""
    eng, ocfg, st, buf, nrm, _ = make_pair(act="tanh", hidden=(64, 96, 48), B=64, seed=41, normalizers="random",
                                           use_expert=True, model_hidden=(80, 64, 96, 48), ne=12,
                                           wm=dict(critic_hidden=(72,)))
    S, A = ocfg.S, ocfg.A
    s, a, _ = _rows(1500, S, A, 1)
    rs = np.random.RandomState(19)
    eng.rng_set_state(rs.get_state())
    pi, nlp = [t.cpu().numpy() for t in eng.evaluate(s)]
    rpi, rnlp = O.actor_evaluate(st, ocfg, nrm, s, rs)
    assert relerr(pi, rpi) < 2e-5 and relerr(nlp, rnlp) < 2e-5
    got = np.asarray(eng.act_host(s[:3], False)).reshape(3, A)      # the GEMM path (not the 2-layer rows kernel)
    o, _ = O.actor_forward(st.actor, O._norm(s[:3].astype(np.float64), nrm.s_mean, nrm.s_den), ocfg)
    mu, lraw = O.split_head(o, st.logstd, ocfg)
    ref_a = O.head_sample(mu, lraw, O.f32_noise(rs.normal(size=mu.shape)), ocfg.act_limit, np.float64)[0]
    assert relerr(got, ref_a) < 2e-5
    assert _same_stream(eng, rs)
    for net, params in (("q0", st.q[0]), ("t1", st.q_targ[1])):
        f = eng.critic_forward(net, s, a).cpu().numpy()
        v = eng.critic_forward(net, s, a, value=True).cpu().numpy()
        assert relerr(f, O.critic_forward(params, ocfg, nrm, s, a)) < 2e-5
        assert relerr(v, O.critic_forward(params, ocfg, nrm, s, a, value=True)) < 2e-5
    for k in range(2):
        pred, sp, r = [t.cpu().numpy() for t in eng.model_forward(k, s, a)]
        rp, rsp, rr = O.model_forward(st, ocfg, nrm, k, s, a)
        assert relerr(pred, rp) < 2e-5 and relerr(sp, rsp) < 2e-5 and relerr(r, rr) < 2e-5
    eng.close()


@pytest.mark.parametrize("deterministic", [False, True])
def test_rollout_any_depth(gpu_available, deterministic):
    eng, ocfg, st, buf, nrm, _ = make_pair(act="relu", hidden=(64, 48, 64), B=64, seed=51, use_expert=True,
                                           normalizers="random", model_hidden=(96,), ne=12, num_models=3)
    s0 = (np.random.RandomState(5).normal(size=(300, ocfg.S)) * 1.5).astype(np.float32)
    eng.rng_set_state(np.random.RandomState(23).get_state())
    ref_rs = np.random.RandomState(23)
    got = [t.cpu().numpy() for t in eng.rollout(2, s0, 4, deterministic)]
    ref = O.rollout(st, ocfg, nrm, s0, 4, 2, ref_rs, deterministic)
    for g, r, name in zip(got[:4], ref[:4], ("s", "a", "r", "sp")):
        assert relerr(g, r) < 1e-4, (name, relerr(g, r))
    assert _same_stream(eng, ref_rs)
    eng.close()


@pytest.mark.parametrize("nm,gauss,use_expert_actions", [(3, False, False), (4, True, False), (5, False, True)])
def test_expert_diag_many_models(gpu_available, nm, gauss, use_expert_actions):
    """model_MSE_on_expert_data / _counterfactual_action averaged over every model (SAC_expert.py:
    579-608) and _calc_disc (:427-460: every model samples -- GaussianModels draw -- and models 0 / 1
    are compared), with nm world models of 3 hidden layers."""
    eng, ocfg, st, buf, nrm, _ = make_pair(act="relu", hidden=(64, 64), B=64, seed=71, use_expert=True,
                                           normalizers="random", model_hidden=(64, 80, 48), ne=12, num_models=nm,
                                           wm=dict(gaussian_model=gauss) if gauss else None)
    S, A, n = ocfg.S, ocfg.A, 300
    r = np.random.RandomState(9)
    s_e = (r.normal(size=(n, S)) * 2).astype(np.float32)
    a_e = r.uniform(-1, 1, (n, A)).astype(np.float32)
    sp_e = (s_e + r.normal(size=(n, S)) * 0.1).astype(np.float32)
    eng.rng_set_state(np.random.RandomState(29).get_state())
    rs = np.random.RandomState(29)
    got = eng.expert_diag(s_e, a_e, sp_e, use_expert_actions=use_expert_actions)
    m_data, m_cf, per_data, per_cf = O.expert_mse_diag(st, ocfg, nrm, s_e, a_e, sp_e, rs, use_expert_actions)
    assert len(got["mse_expert_data_per_model"]) == nm
    assert abs(got["mse_expert_data"] - m_data) <= 1e-4 * abs(m_data)
    assert abs(got["mse_counterfactual"] - m_cf) <= 1e-4 * abs(m_cf)
    assert np.max(np.abs(got["mse_expert_data_per_model"] - per_data) / np.abs(per_data)) < 1e-4
    got_d = eng.expert_diag(s_e, a_e, sp_e, disc=True, use_expert_actions=use_expert_actions)
    ratio, mx, med, tot = O.calc_disc(st, ocfg, nrm, s_e, a_e, rs, use_expert_actions)
    assert abs(got_d["s_disc_total"] - tot) <= 1e-4 * tot
    assert abs(got_d["max_disc"] - mx) <= 1e-4 * mx
    assert relerr(got_d["disc_ratio"], ratio) < 1e-4
    assert _same_stream(eng, rs)
    eng.close()


def test_generic_plan_is_taken(gpu_available, monkeypatch):
    """The plan a deep handle runs: every hidden layer its own forward problem, the row-kernel heads
    (k_actor_head / k_qhead / k_actor_bwd), no fused launch names; the default depth keeps the fused
    plan (8 launches per update for plain SAC)."""
    eng, *_ = _pair(monkeypatch, "actor3")
    names = [p["name"] for p in eng.plan_info()]
    for n in ("actor.fwd0", "actor.fwd1", "actor.fwd2", "actor.head", "q.head", "pi.q.head", "actor.head.bwd",
              "actor.bwd2", "actor.bwd1", "actor.adam", "critic.adam", "alpha.final"):
        assert n in names, (n, names)
    assert not any("+" in n for n in names), names
    eng.close()
    eng, *_ = make_pair(hidden=(64, 64), B=64, seed=1)
    names = [p["name"] for p in eng.plan_info()]
    assert "q.fwd01+actor.head" in names and "actor.head" not in names, names
    eng.close()
