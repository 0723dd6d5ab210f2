"""The world-model variants on the device, each against the oracle:

* --gaussian_model: GaussianModel (continuous_models.py:7-201) -- a trainable logstd [1, S] per
  model fitted by the Gaussian NLL (:101-131) in the same model-optimiser step as the net, with
  --scale_model_loss's stop-gradient mean(exp(2 logstd)) (:122-127); sample(deterministic=False)
  and step add exp(logstd) * u, u = np.random.normal(size=(n, S)) from the global stream (:36-70);
  the SAC-EO expert term samples deterministically (SAC_expert.py:291, :325-326).
* --separate_reward_nn (base_world_model.py:32-37, :72-74): the model net predicts the S deltas, a
  reward net [S+A] -> reward_layers -> 1 the reward, fitted in the same step.

Compared: one SAC-EO update (losses within 2e-5), model-fit steps eager and graph (losses within
1e-4, every weight incl. logstd and the reward nets within 5e-5 after 5 steps, with and without the
global-norm clip and the loss clips), the reference objects' forward / sample / step / get_loss,
the rollout and the _calc_disc diagnostics (the device stream bit-exact after each)."""
import numpy as np
import pytest

import sac_oracle as O
from helpers import make_pair, oracle_step, relerr

pytestmark = pytest.mark.gpu

VARIANTS = {
    "gauss": dict(gaussian_model=True),
    "gauss_scale": dict(gaussian_model=True, scale_model_loss=True),
    "reward_nn": dict(separate_reward_nn=True, reward_hidden=(96, 64), reward_act="tanh"),
    "gauss_reward_scale": dict(gaussian_model=True, scale_model_loss=True, separate_reward_nn=True,
                               reward_hidden=(64, 80), reward_act="elu"),
}


def _same_stream(eng, rs):
    dev, ref = eng.rng_get_state(), rs.get_state()
    return np.array_equal(dev[1], ref[1]) and dev[2] == ref[2] and dev[3] == ref[3] and dev[4] == ref[4]


def _rows(n, S, A, seed=0):
    r = np.random.RandomState(seed)
    s = (r.normal(size=(n, S)) * 1.5).astype(np.float32)
    a = r.uniform(-1, 1, (n, A)).astype(np.float32)
    sp = (s + r.normal(size=(n, S)) * 0.3).astype(np.float32)
    rr = r.normal(size=n).astype(np.float32)
    return s, a, sp, rr


@pytest.mark.parametrize("variant", list(VARIANTS))
def test_update_with_model_variant(gpu_available, variant):
    """One SAC-EO update: the expert term samples the world models deterministically, through
    the S delta columns of the model net (S + 1 or S wide)."""
    B, ne = 128, 12
    eng, ocfg, st, buf, nrm, expert = make_pair(act="relu", B=B, seed=23, use_expert=True, ne=ne,
                                                normalizers="random", model_hidden=(96, 128), wm=VARIANTS[variant])
    N = buf["r"].shape[0]
    rs = np.random.RandomState(92)
    eng.rng_set_state(rs.get_state())
    gen = np.random.default_rng(5)
    R = O.draw_step_randoms(rs, N, B, ocfg.A, n_expert=ne, gen=gen)
    eng.push_perms(R["perm"][None])
    ref = oracle_step(st, ocfg, nrm, buf, R, expert)
    eng.step(1, eager=True)
    eng.sync()
    row = eng.stats(1)[0]
    for i, k in enumerate(("q1_loss", "q2_loss", "p_loss", "alpha_loss")):
        assert abs(row[i] - ref[k]) <= 2e-5 * abs(ref[k]) + 1e-7, (k, row[i], ref[k])
    assert abs(row[5] - ref["mse_loss"]) <= 2e-5 * abs(ref["mse_loss"])
    assert _same_stream(eng, rs)
    eng.close()


@pytest.mark.parametrize("variant,nm,max_norm,dclip", [
    ("gauss", 2, 0.0, 0.0), ("gauss_scale", 2, 0.0, 0.3), ("reward_nn", 2, 0.0, 0.0),
    ("gauss_reward_scale", 2, 0.05, 0.0), ("gauss", 1, 0.02, 0.0), ("reward_nn", 1, 0.0, 0.2)])
def test_model_fit_variant(gpu_available, variant, nm, max_norm, dclip):
    """sacx_model_fit with GaussianModels / reward nets: 2 eager steps, then 3 graph-replayed ones;
    the summed loss of every step and every model variable (net, logstd, reward net) against
    O.model_fit_step (the logstd Adam in the fit's finalisation, or the global-norm clip over the
    models' whole variable range)."""
    eng, ocfg, st, buf, nrm, _ = make_pair(act="relu", B=64, seed=33, use_expert=True, normalizers="random",
                                           num_models=nm, model_max_grad_norm=max_norm, delta_clip_loss=dclip,
                                           model_hidden=(128, 96), wm=VARIANTS[variant])
    N = buf["r"].shape[0]
    mb = eng.cfg.model_batch
    idx = np.random.RandomState(13).randint(N, size=(5, nm, mb))
    for eager in (True, False):
        eng.model_fit(idx[:2] if eager else idx[2:], eager=eager)
    eng.sync()
    dev = eng.model_stats(5)
    ref = []
    for j in range(5):
        batches = [(buf["s"][idx[j, k]], buf["a"][idx[j, k]], buf["sp"][idx[j, k]], buf["r"][idx[j, k]])
                   for k in range(nm)]
        ref.append(O.model_fit_step(st, ocfg, nrm, batches, max_grad_norm=max_norm or None, delta_clip_loss=dclip))
    ref = np.array(ref)
    assert np.max(np.abs(dev - ref) / np.abs(ref)) < 1e-4, (dev, ref)
    for k in range(nm):
        for a_, b_ in zip(eng.get_net(f"m{k}"), st.models[k]):
            assert np.max(np.abs(a_ - b_)) < 5e-5
        if ocfg.gaussian_model:
            got = eng.get_model_logstd(k)
            assert np.max(np.abs(got - st.model_logstd[k])) < 5e-5, (got, st.model_logstd[k])
            init = O.init_state(ocfg, seed=34, with_models=True, model_std_mult=0.7).model_logstd[k]
            assert not np.allclose(got, init)          # trained
        if ocfg.separate_reward_nn:
            for a_, b_ in zip(eng.get_net(f"r{k}"), st.reward_nets[k]):
                assert np.max(np.abs(a_ - b_)) < 5e-5
    eng.close()


def test_reset_model_optimizer_every_model_trainable(gpu_available):
    """--reset_model_optimizer (SAC_expert.py:553-555) builds a fresh Keras Adam: no moment survives
    for any model trainable -- the model nets, GaussianModel's logstd AND the separate reward nets.
    Fit 2 steps, reset, fit 2 more: every variable against the oracle with a fresh AdamState."""
    eng, ocfg, st, buf, nrm, _ = make_pair(act="relu", B=64, seed=35, use_expert=True, normalizers="random",
                                           num_models=2, model_hidden=(96, 64), wm=VARIANTS["gauss_reward_scale"])
    N = buf["r"].shape[0]
    mb = eng.cfg.model_batch
    idx = np.random.RandomState(17).randint(N, size=(4, 2, mb))
    dev = []
    for half in (0, 1):
        eng.model_fit(idx[2 * half: 2 * half + 2], eager=True)
        if half == 0:
            eng.reset_model_optimizer()
    eng.sync()
    dev = eng.model_stats(4)
    ref = []
    for j in range(4):
        if j == 2:
            st.opt_model = O.AdamState.zeros_like(st.model_all_vars())
        batches = [(buf["s"][idx[j, k]], buf["a"][idx[j, k]], buf["sp"][idx[j, k]], buf["r"][idx[j, k]])
                   for k in range(2)]
        ref.append(O.model_fit_step(st, ocfg, nrm, batches))
    ref = np.array(ref)
    assert np.max(np.abs(dev - ref) / np.abs(ref)) < 1e-4, (dev, ref)
    for k in range(2):
        for a_, b_ in zip(eng.get_net(f"m{k}"), st.models[k]):
            assert np.max(np.abs(a_ - b_)) < 5e-5
        assert np.max(np.abs(eng.get_model_logstd(k) - st.model_logstd[k])) < 5e-5
        for a_, b_ in zip(eng.get_net(f"r{k}"), st.reward_nets[k]):
            assert np.max(np.abs(a_ - b_)) < 5e-5
    eng.close()


@pytest.mark.parametrize("variant", ["gauss", "gauss_reward_scale", "reward_nn"])
def test_model_forward_sample_loss(gpu_available, variant):
    """_forward / sample(deterministic and not) / get_loss on the device vs the oracle; the
    stochastic sample draws normal(size=(n, S)) (GaussianModel), the deterministic one nothing;
    n crosses the 4,096-row chunk."""
    eng, ocfg, st, buf, nrm, _ = make_pair(act="relu", B=64, seed=45, use_expert=True, normalizers="random",
                                           model_hidden=(96, 96), wm=VARIANTS[variant])
    nrm.r_mean, nrm.r_den = np.float32(0.3), np.float32(1.7)
    eng.set_normalizers(nrm.s_mean, nrm.s_den, nrm.a_mean, nrm.a_den, nrm.d_mean, nrm.d_den,
                        nrm.r_mean, nrm.r_den, nrm.ret_den)
    for n in (1, 300, 5000):
        s, a, sp, r = _rows(n, ocfg.S, ocfg.A, 3)
        for k in range(2):
            pred, spd, rd = [t.cpu().numpy() for t in eng.model_forward(k, s, a, 0.05, 0.3)]
            rp, rsp, rr = O.model_forward(st, ocfg, nrm, k, s, a, 0.05, 0.3)
            assert relerr(pred, rp) < 2e-5 and relerr(spd, rsp) < 2e-5 and relerr(rd, rr) < 2e-5
            eng.rng_set_state(np.random.RandomState(40 + k).get_state())
            rs = np.random.RandomState(40 + k)
            _, spn, _ = [t.cpu().numpy() for t in eng.model_forward(k, s, a, 0.0, 0.0, stochastic=True)]
            u = rs.normal(size=(n, ocfg.S)) if ocfg.gaussian_model else None
            _, rspn, _ = O.model_forward(st, ocfg, nrm, k, s, a, noise=u)
            assert relerr(spn, rspn) < 2e-5 and _same_stream(eng, rs)
            got = eng.model_loss(k, s, sp, a, r, 0.5, 1.0)
            ref = O.model_loss(st, ocfg, nrm, k, s, sp, a, r, 0.5, 1.0)
            assert abs(got - ref) <= 1e-5 * abs(ref), (k, n, got, ref)
    eng.close()


@pytest.mark.parametrize("variant,deterministic", [("gauss", False), ("gauss_reward_scale", True),
                                                   ("reward_nn", False)])
def test_rollout_variant(gpu_available, variant, deterministic):
    """batch_simtrajectory_sampler over GaussianModel.step (always noisy: the actor's (n, A) draw,
    then the model's (n, S), per step) / a model with a reward net: trajectories within 1e-4, the
    stream bit-exact."""
    eng, ocfg, st, buf, nrm, _ = make_pair(act="tanh", B=64, seed=51, use_expert=True, normalizers="random",
                                           model_hidden=(64, 64), wm=VARIANTS[variant])
    s0 = (np.random.RandomState(5).normal(size=(300, ocfg.S)) * 1.5).astype(np.float32)
    eng.rng_set_state(np.random.RandomState(23).get_state())
    rs = np.random.RandomState(23)
    got = [t.cpu().numpy() for t in eng.rollout(1, s0, 4, deterministic)]
    ref = O.rollout(st, ocfg, nrm, s0, 4, 1, rs, deterministic)
    for g, r, name in zip(got, ref, ("s", "a", "r", "sp", "d")):
        assert g.shape == r.shape, (name, g.shape, r.shape)
        if name != "d":
            assert relerr(g, r) < 1e-4, (name, relerr(g, r))
    assert _same_stream(eng, rs)
    eng.close()


@pytest.mark.parametrize("use_expert_actions", [False, True])
def test_disc_diag_gaussian(gpu_available, use_expert_actions):
    """_calc_disc with GaussianModels (SAC_expert.py:427-460: model.sample(deterministic=False)):
    the counterfactual action's draw, then model 0's and model 1's (n, S) noise; the MSE
    diagnostics (deterministic samples) draw only the counterfactual action."""
    eng, ocfg, st, buf, nrm, _ = make_pair(act="relu", B=64, seed=71, use_expert=True, normalizers="random",
                                           model_hidden=(64, 64), wm=VARIANTS["gauss_reward_scale"])
    S, A, n = ocfg.S, ocfg.A, 40
    r = np.random.RandomState(9)
    s_e = (r.normal(size=(n, S)) * 2).astype(np.float32)
    a_e = r.uniform(-1, 1, (n, A)).astype(np.float32)
    sp_e = (s_e + r.normal(size=(n, S)) * 0.1).astype(np.float32)
    eng.rng_set_state(np.random.RandomState(29).get_state())
    rs = np.random.RandomState(29)
    got = eng.expert_diag(s_e, a_e, sp_e, use_expert_actions=use_expert_actions)
    m_data, m_cf, _, _ = O.expert_mse_diag(st, ocfg, nrm, s_e, a_e, sp_e, rs, use_expert_actions)
    assert abs(got["mse_expert_data"] - m_data) <= 1e-4 * abs(m_data)
    assert abs(got["mse_counterfactual"] - m_cf) <= 1e-4 * abs(m_cf)
    got_d = eng.expert_diag(s_e, a_e, sp_e, disc=True, use_expert_actions=use_expert_actions)
    ratio, mx, med, tot = O.calc_disc(st, ocfg, nrm, s_e, a_e, rs, use_expert_actions)
    assert abs(got_d["s_disc_total"] - tot) <= 1e-4 * tot
    assert abs(got_d["max_disc"] - mx) <= 1e-4 * mx
    assert relerr(got_d["disc_ratio"], ratio) < 1e-4
    assert _same_stream(eng, rs)
    eng.close()


def test_reference_objects_gaussian_and_reward_net(gpu_available):
    """init_world_models(gaussian_model=True) with --separate_reward_nn: GaussianModel objects whose
    get_weights / set_weights carry [net..., logstd] and get_reward_weights the reward net, whose
    sample / step / get_loss / entropy return what the reference's do (through the device)."""
    from sac_eo.common.train_parser import create_train_parser, gather_inputs
    from sac_eo.envs import init_env
    from sac_eo.models import GaussianModel, init_world_models
    eng, ocfg, st, buf, nrm, _ = make_pair(act="relu", B=64, seed=49, use_expert=True, model_hidden=(96, 96),
                                           wm=VARIANTS["gauss_reward_scale"])
    env = init_env("gym", "HalfCheetah-v3")
    k = gather_inputs(create_train_parser().parse_args(
        ["--gaussian_model", "--separate_reward_nn", "--scale_model_loss", "--model_layers", "96", "96",
         "--reward_layers", "64", "80", "--reward_activations", "elu", "--model_std_mult", "0.5"]))
    models = init_world_models(env, **dict(k["model_kwargs"], model_weights=None, reward_weights=None),
                               model_setup_kwargs=k["model_setup_kwargs"])
    m = models[1]
    assert isinstance(m, GaussianModel) and m.separate_reward_nn
    w = m.get_weights()
    assert len(w) == 7 and w[-1].shape == (1, ocfg.S) and np.allclose(w[-1], np.log(0.5))
    assert w[4].shape == (96, ocfg.S)                      # the model net predicts the deltas only
    m.set_weights(st.models[1] + [st.model_logstd[1]])
    m.set_reward_weights(st.reward_nets[1])
    m._bind(eng, "m1")
    assert np.allclose(m.get_weights()[-1], st.model_logstd[1])
    assert all(np.allclose(x, y) for x, y in zip(m.get_reward_weights(), st.reward_nets[1]))
    s, a, sp, r = _rows(5, ocfg.S, ocfg.A, 5)
    _, rsp, rr = O.model_forward(st, ocfg, nrm, 1, s, a)
    assert relerr(m.sample(s, a, deterministic=True), rsp) < 2e-5
    eng.rng_set_state(np.random.RandomState(3).get_state())
    rs = np.random.RandomState(3)
    m.reset(s)
    s1, r1, d1, _ = m.step(a)                              # GaussianModel.step: noisy
    _, rsp1, rr1 = O.model_forward(st, ocfg, nrm, 1, s, a, noise=rs.normal(size=(5, ocfg.S)))
    assert relerr(s1, rsp1) < 2e-5 and relerr(r1, rr1) < 2e-5 and not np.any(d1)
    assert _same_stream(eng, rs)
    loss = m.get_loss(s, sp, a, r)
    assert abs(loss - O.model_loss(st, ocfg, nrm, 1, s, sp, a, r)) <= 1e-5 * abs(loss)
    ent = m.entropy(s, a)
    assert ent.shape == (5,) and abs(ent[0] - O.model_entropy(st, ocfg, 1)) < 1e-5
    eng.close()
