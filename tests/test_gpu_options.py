"""Reference options on the device path, each against the oracle:

* --num_models 1 (SAC_expert.py:273-296): the expert term through one world model on every
  expert row in order (no shuffle), the mean MSE over the rows; one update per stage and a
  100-update trajectory on the production schedule; the model fit of one model.
* --model_max_grad_norm (mbrl_onpolicy_alg.py:315-317: clip_by_global_norm to
  max_norm * num_models) and --delta_clip_loss / --reward_clip_loss
  (continuous_models.py:284-296) in the model fit.
* GaussianActor.sample (continuous_actors.py:74-123, an expert imported from a log:
  train.py:65-86 builds it without actor_squash), ± per_state_std, ± output_norm.
"""
import numpy as np
import pytest

import sac_oracle as O
from helpers import make_pair, oracle_step, relerr

pytestmark = pytest.mark.gpu


def test_one_model_update_matches_oracle(gpu_available):
    B, ne = 128, 15                      # one model: an odd expert batch is allowed
    eng, ocfg, st, buf, nrm, expert = make_pair(act="relu", B=B, seed=17, use_expert=True, ne=ne,
                                                normalizers="random", done_p=0.02, num_models=1)
    N = buf["r"].shape[0]
    rs = np.random.RandomState(90)
    eng.rng_set_state(rs.get_state())
    R = O.draw_step_randoms(rs, N, B, ocfg.A, n_expert=ne, n_models=1)
    keep = {}
    ref = oracle_step(st, ocfg, nrm, buf, R, expert, keep)
    eng.step(1, eager=True)
    eng.sync()
    row = eng.stats(1)[0]
    for i, k in enumerate(("q1_loss", "q2_loss", "p_loss", "alpha_loss")):
        assert abs(row[i] - ref[k]) <= 2e-5 * abs(ref[k]) + 1e-7, (k, row[i], ref[k])
    assert abs(row[5] - ref["mse_loss"]) <= 2e-5 * abs(ref["mse_loss"])
    m = eng.v["adam_m"][0]
    for i in range(3):
        seg = eng.segments[f"actor.l{i}"]
        o, n = seg["offset"] // 4, seg["rows"] * seg["cols"]
        gd = m[o:o + n].cpu().numpy().reshape(seg["rows"], seg["cols"]) / (np.float32(1) - np.float32(0.9))
        assert relerr(gd[:-1], keep["actor_grads"][2 * i]) < 2e-4
        assert relerr(gd[-1], keep["actor_grads"][2 * i + 1]) < 2e-4
    got, exp = eng.rng_get_state(), rs.get_state()
    assert np.array_equal(got[1], exp[1]) and got[2] == exp[2] and got[3] == exp[3]
    eng.close()


def test_one_model_trajectory(gpu_available):
    B, ne, steps = 256, 20, 100
    eng, ocfg, st, buf, nrm, expert = make_pair(act="relu", B=B, seed=19, use_expert=True, ne=ne, done_p=0.01,
                                                graph_steps=128, num_models=1)
    N = buf["r"].shape[0]
    rs = np.random.RandomState(91)
    eng.rng_set_state(rs.get_state())
    Rs = [O.draw_step_randoms(rs, N, B, ocfg.A, n_expert=ne, n_models=1) for _ in range(steps)]
    eng.prepare(steps)
    eng.step(steps)
    eng.sync()
    dev = eng.stats(steps)
    ref = np.array([[o["q1_loss"], o["q2_loss"], o["p_loss"], o["mse_loss"]]
                    for o in (oracle_step(st, ocfg, nrm, buf, R, expert) for R in Rs)])
    assert np.max(np.abs(dev[:, :2] - ref[:, :2]) / np.abs(ref[:, :2])) < 1e-4
    assert np.max(np.abs(dev[:, 2] - ref[:, 2])) / np.max(np.abs(ref[:, 2])) < 1e-4
    assert np.max(np.abs(dev[:, 5] - ref[:, 3]) / np.abs(ref[:, 3])) < 1e-4
    eng.close()


@pytest.mark.parametrize("nm,max_norm,dclip,rclip", [(2, 0.05, 0.0, 0.0), (1, 0.0, 0.0, 0.0),
                                                     (1, 0.02, 0.3, 0.5), (2, 0.0, 0.2, 0.0)])
def test_model_fit_options(gpu_available, nm, max_norm, dclip, rclip):
    eng, ocfg, st, buf, nrm, _ = make_pair(act="relu", B=64, seed=31, use_expert=True, normalizers="random",
                                           num_models=nm, model_max_grad_norm=max_norm, delta_clip_loss=dclip,
                                           reward_clip_loss=rclip)
    N = buf["r"].shape[0]
    mb = eng.cfg.model_batch
    idx = np.random.RandomState(12).randint(N, size=(5, nm, mb))
    for eager in (True, False):
        eng.model_fit(idx[:2] if eager else idx[2:], eager=eager)
    eng.sync()
    dev = eng.model_stats(5)
    ref = []
    for j in range(5):
        batches = [(buf["s"][idx[j, k]], buf["a"][idx[j, k]], buf["sp"][idx[j, k]], buf["r"][idx[j, k]])
                   for k in range(nm)]
        ref.append(O.model_fit_step(st, ocfg, nrm, batches, max_grad_norm=max_norm or None,
                                    delta_clip_loss=dclip, reward_clip_loss=rclip))
    ref = np.array(ref)
    assert np.max(np.abs(dev - ref) / np.abs(ref)) < 1e-4, (dev, ref)
    for k in range(nm):
        for a_, b_ in zip(eng.get_net(f"m{k}"), st.models[k]):
            assert np.max(np.abs(a_ - b_)) < 5e-5
    eng.close()


@pytest.mark.parametrize("per_state_std,output_norm,deterministic,n", [(False, False, True, 300), (False, True, False, 300),
                                                                       (True, False, False, 300), (True, True, True, 300),
                                                                       (True, True, False, 1), (False, True, True, 16)])
def test_gaussian_actor_sample(gpu_available, per_state_std, output_norm, deterministic, n):
    """n <= 16 rows take k_act_rows (one workgroup per row), n = 300 the batched launches."""
    from sac_eo.engine import Engine, EngineConfig
    S, A = 11, 3
    cfg = O.Config(S=S, A=A, hidden=(64, 64), act="tanh", per_state_std=per_state_std)
    st = O.init_state(cfg, seed=8, bias_scale=0.2, actor_gain=2.0)
    st.logstd = np.full((1, A), -0.7, np.float32)
    eng = Engine(EngineConfig(s_dim=S, a_dim=A, hidden=(64, 64), activation="tanh", batch=1, buffer_capacity=1,
                              per_state_std=per_state_std, graph_steps=1, actor_gaussian=True, actor_std_mult=0.6,
                              actor_output_norm=output_norm))
    eng.set_net("actor", st.actor)
    eng.set_logstd(st.logstd)
    nrm = O.Normalizers.identity(S, A)
    obs = (np.random.RandomState(4).normal(size=(n, S)) * 2).astype(np.float32)
    eng.rng_set_state(np.random.RandomState(7).get_state())
    rs = np.random.RandomState(7)
    got = eng.act(obs, deterministic=deterministic).cpu().numpy()
    u = np.zeros((n, A)) if deterministic else O.f32_noise(rs.normal(size=(n, A))).astype(np.float64)
    ref = O.gaussian_actor_sample([w.astype(np.float64) for w in st.actor], st.logstd.astype(np.float64), cfg, nrm,
                                  obs, u, 0.6, output_norm)
    assert relerr(got, ref) < 2e-5, relerr(got, ref)
    if output_norm:                         # the mean is normalised: |a| is not squashed below 1
        assert np.all(np.isfinite(got))
    with pytest.raises(Exception):
        eng.step(1)                         # inference only
    eng.close()


def _actor_grads(eng, B1):
    """The actor's gradients read back through Adam's first moment (m_1 = g (1 - beta1)), in
    the Keras weight-list order (with the layer norm: [W0, b0, gamma, beta, W1, b1, W2, b2])."""
    m = eng.v["adam_m"][0]
    out = []
    for i in range(3):
        seg = eng.segments[f"actor.l{i}"]
        o, n = seg["offset"] // 4, seg["rows"] * seg["cols"]
        w = m[o:o + n].cpu().numpy().reshape(seg["rows"], seg["cols"]) / B1
        out += [w[:-1], w[-1]]
        if i == 0 and "actor.ln" in eng.segments:
            seg = eng.segments["actor.ln"]
            o = seg["offset"] // 4
            gb = m[o:o + 2 * seg["cols"]].cpu().numpy().reshape(2, -1) / B1
            out += [gb[0], gb[1]]
    return out


@pytest.mark.parametrize("use_expert", [False, True])
def test_layer_norm_update_matches_oracle(gpu_available, use_expert):
    """--actor_layer_norm: one update per stage vs the oracle, gamma / beta gradients included."""
    B = 128
    eng, ocfg, st, buf, nrm, expert = make_pair(act="relu", B=B, seed=23, use_expert=use_expert, layer_norm=True,
                                                normalizers="random", done_p=0.02)
    N = buf["r"].shape[0]
    rs = np.random.RandomState(93)
    gen = np.random.default_rng(94)
    eng.rng_set_state(rs.get_state())
    R = O.draw_step_randoms(rs, N, B, ocfg.A, n_expert=20 if use_expert else 0, gen=gen)
    if use_expert:
        eng.push_perms(R["perm"][None, :])
    keep = {}
    ref = oracle_step(st, ocfg, nrm, buf, R, expert, keep)
    eng.step(1, eager=True)
    eng.sync()
    row = eng.stats(1)[0]
    for i, k in enumerate(("q1_loss", "q2_loss", "p_loss", "alpha_loss")):
        assert abs(row[i] - ref[k]) <= 2e-5 * abs(ref[k]) + 1e-7, (k, row[i], ref[k])
    got = _actor_grads(eng, np.float32(1) - np.float32(0.9))
    assert len(got) == 8
    for gd, go in zip(got, keep["actor_grads"]):
        assert relerr(gd, go) < 2e-4, relerr(gd, go)
    eng.close()


@pytest.mark.parametrize("use_expert", [False, True])
def test_layer_norm_trajectory_and_graph(gpu_available, use_expert):
    """100 updates on the production schedule (the alpha rows' layer norm folded into the next
    update's) vs the oracle, and graph replay == eager launches bit for bit."""
    B, steps = 128, 100
    outs = []
    for eager in (False, True):
        eng, ocfg, st, buf, nrm, expert = make_pair(act="tanh", B=B, seed=25, use_expert=use_expert, layer_norm=True,
                                                    done_p=0.01, graph_steps=128)
        N = buf["r"].shape[0]
        rs = np.random.RandomState(95)
        gen = np.random.default_rng(96)
        eng.rng_set_state(rs.get_state())
        Rs = [O.draw_step_randoms(rs, N, B, ocfg.A, n_expert=20 if use_expert else 0, gen=gen) for _ in range(steps)]
        if use_expert:
            eng.push_perms(np.stack([R["perm"] for R in Rs]))
        eng.step(steps, eager=eager)
        eng.sync()
        outs.append((eng.stats(steps).copy(), eng.v["params"].cpu().numpy().copy()))
        eng.close()
    ref = np.array([[o["q1_loss"], o["q2_loss"], o["p_loss"]] for o in (oracle_step(st, ocfg, nrm, buf, R, expert)
                                                                        for R in Rs)])
    dev = outs[0][0]
    assert np.max(np.abs(dev[:, :2] - ref[:, :2]) / np.abs(ref[:, :2])) < 1e-4
    assert np.max(np.abs(dev[:, 2] - ref[:, 2])) / np.max(np.abs(ref[:, 2])) < 1e-4
    assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])


def test_layer_norm_inference_paths(gpu_available):
    """sample / evaluate / rollout through the layer-norm actor."""
    eng, ocfg, st, buf, nrm, _ = make_pair(act="relu", B=64, seed=27, use_expert=True, layer_norm=True,
                                           normalizers="random")
    s = (np.random.RandomState(2).normal(size=(50, ocfg.S)) * 1.5).astype(np.float32)
    eng.rng_set_state(np.random.RandomState(11).get_state())
    rs = np.random.RandomState(11)
    pi, nlp = [t.cpu().numpy() for t in eng.evaluate(s)]
    rpi, rnlp = O.actor_evaluate(st, ocfg, nrm, s, rs)
    assert relerr(pi, rpi) < 2e-5 and relerr(nlp, rnlp) < 2e-5
    got = [t.cpu().numpy() for t in eng.rollout(0, s, 3)]
    ref = O.rollout(st, ocfg, nrm, s, 3, 0, rs)
    for g, r, name in zip(got, ref, ("s", "a", "r", "sp", "d")):
        if name != "d":
            assert relerr(g, r) < 1e-4, name
    eng.close()


@pytest.mark.parametrize("nm,dcp", [(1, 0.2), (2, 0.1)])
def test_delta_clip_pred_update(gpu_available, nm, dcp):
    """--delta_clip_pred in the SAC-EO expert term (MSEModel.sample -> _forward(clip=True),
    base_world_model.py:80-82): the clipped prediction enters the MSE and its gradient is zero
    outside [-c, c] (tf.clip_by_value).  c is chosen so that a part of the predictions clip."""
    B, ne = 128, 20
    eng, ocfg, st, buf, nrm, expert = make_pair(act="relu", B=B, seed=23, use_expert=True, ne=ne,
                                                normalizers="random", num_models=nm, delta_clip_pred=dcp)
    ocfg.delta_clip_pred = dcp
    N = buf["r"].shape[0]
    rs = np.random.RandomState(92)
    eng.rng_set_state(rs.get_state())
    R = O.draw_step_randoms(rs, N, B, ocfg.A, n_expert=ne, n_models=nm, gen=np.random.default_rng(29))
    if nm == 2:
        eng.push_perms(R["perm"][None, :])
    keep = {}
    ref = oracle_step(st, ocfg, nrm, buf, R, expert, keep)
    frac = np.mean([keep["clip_frac%d" % k] for k in range(nm)])
    assert 0.05 < frac < 0.95, frac          # both branches of the clip are exercised
    eng.step(1, eager=True)
    eng.sync()
    row = eng.stats(1)[0]
    for i, k in enumerate(("q1_loss", "q2_loss", "p_loss", "alpha_loss")):
        assert abs(row[i] - ref[k]) <= 2e-5 * abs(ref[k]) + 1e-7, (k, row[i], ref[k])
    assert abs(row[5] - ref["mse_loss"]) <= 2e-5 * abs(ref["mse_loss"])
    m = eng.v["adam_m"][0]
    for i in range(3):
        seg = eng.segments[f"actor.l{i}"]
        o, n = seg["offset"] // 4, seg["rows"] * seg["cols"]
        gd = m[o:o + n].cpu().numpy().reshape(seg["rows"], seg["cols"]) / (np.float32(1) - np.float32(0.9))
        assert relerr(gd[:-1], keep["actor_grads"][2 * i]) < 2e-4
        assert relerr(gd[-1], keep["actor_grads"][2 * i + 1]) < 2e-4
    eng.close()


@pytest.mark.parametrize("chid,use_expert", [((96, 48), False), ((400, 300), False), ((64, 128), True)])
def test_critic_hidden_sizes(gpu_available, chid, use_expert):
    """--critic_layers different from --actor_layers (nn_utils.py:86-138 builds each net from its own
    list; train_parser.py:56-59, :80-84): one update per stage against the oracle, then 19 graph-replayed
    updates equal to eager launches bit for bit."""
    B = 128
    ne = 12 if use_expert else 20
    eng, ocfg, st, buf, nrm, expert = make_pair(act="relu", B=B, seed=29, use_expert=use_expert, ne=ne,
                                                normalizers="random", model_hidden=(64, 64), wm=dict(critic_hidden=chid))
    assert eng.segments["q0.l0"]["cols"] == chid[0] and eng.segments["t1.l1"]["cols"] == chid[1]
    N = buf["r"].shape[0]
    rs = np.random.RandomState(95)
    eng.rng_set_state(rs.get_state())
    gen = np.random.default_rng(3) if use_expert else None
    R = O.draw_step_randoms(rs, N, B, ocfg.A, n_expert=ne if use_expert else 0, gen=gen)
    if use_expert:
        eng.push_perms(R["perm"][None])
    ref = oracle_step(st, ocfg, nrm, buf, R, expert)
    eng.step(1, eager=True)
    eng.sync()
    row = eng.stats(1)[0]
    for i, k in enumerate(("q1_loss", "q2_loss", "p_loss", "alpha_loss")):
        assert abs(row[i] - ref[k]) <= 2e-5 * abs(ref[k]) + 1e-7, (k, row[i], ref[k])
    for n, nets in (("q0", st.q[0]), ("t1", st.q_targ[1]), ("actor", st.actor)):
        for a_, b_ in zip(eng.get_net(n), nets):
            assert relerr(a_, b_) < 2e-4, n
    eng.close()
    outs = []
    for eager in (True, False):
        eng, *_ = make_pair(act="relu", B=B, seed=29, use_expert=use_expert, ne=ne, normalizers="random",
                            model_hidden=(64, 64), graph_steps=8, wm=dict(critic_hidden=chid))
        eng.rng_set_state(np.random.RandomState(96).get_state())
        if use_expert:
            eng.push_perms(np.stack([np.random.RandomState(j).permutation(ne) for j in range(19)]))
        eng.step(19, eager=eager)
        eng.sync()
        outs.append((eng.stats(19).copy(), eng.v["params"].cpu().numpy().copy()))
        eng.close()
    assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])
