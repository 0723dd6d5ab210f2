"""The reference objects' standalone network calls on the device (the
methods a caller written against the reference's actor / critic / model objects uses), each
through the C ABI and through the reference-named Python objects, against the oracle.

* SquashedGaussianActor.evaluate (continuous_actors.py:327-379): pi and neglogp within 2e-5
  relative to the tensor's max, the device RNG stream advanced exactly as the reference's
  np.random.normal(size=(n, A)).
* QCritic._forward / value (critics.py:84-103), q_critics and q_targets: within 2e-5.
* MSEModel._forward / sample / step / get_loss (continuous_models.py:225-302,
  base_world_model.py:65-87), with and without the prediction / loss clips: within 2e-5 (the
  loss: 1e-5 relative).
Row counts cross the workspace chunks (1,024 rows per critic / actor chunk, 4,096 per model
chunk) and include n = 1.
"""
import numpy as np
import pytest

import sac_oracle as O
from helpers import make_pair, relerr

pytestmark = pytest.mark.gpu


def _rows(n, S, A, seed=0):
    r = np.random.RandomState(seed)
    s = (r.normal(size=(n, S)) * 1.5).astype(np.float32)
    a = r.uniform(-1, 1, (n, A)).astype(np.float32)
    sp = (s + r.normal(size=(n, S)) * 0.2).astype(np.float32)
    rr = r.normal(size=n).astype(np.float32)
    return s, a, sp, rr


@pytest.mark.parametrize("n,per_state_std", [(37, False), (1, False), (2500, False), (64, True)])
def test_actor_evaluate(gpu_available, n, per_state_std):
    eng, ocfg, st, buf, nrm, _ = make_pair(act="tanh", B=64, seed=41, normalizers="random",
                                           per_state_std=per_state_std)
    s, *_ = _rows(n, ocfg.S, ocfg.A, 1)
    eng.rng_set_state(np.random.RandomState(19).get_state())
    rs = np.random.RandomState(19)
    pi, nlp = [t.cpu().numpy() for t in eng.evaluate(s)]
    rpi, rnlp = O.actor_evaluate(st, ocfg, nrm, s, rs)
    assert relerr(pi, rpi) < 2e-5 and relerr(nlp, rnlp) < 2e-5, (relerr(pi, rpi), relerr(nlp, rnlp))
    dev, ref = eng.rng_get_state(), rs.get_state()
    assert np.array_equal(dev[1], ref[1]) and dev[2] == ref[2] and dev[3] == ref[3] and dev[4] == ref[4]
    eng.close()


@pytest.mark.parametrize("n", [1, 300, 2100])
def test_critic_forward_and_value(gpu_available, n):
    eng, ocfg, st, buf, nrm, _ = make_pair(act="elu", B=64, seed=43, normalizers="random")
    nrm.ret_den = np.float32(2.5)
    eng.set_normalizers(nrm.s_mean, nrm.s_den, nrm.a_mean, nrm.a_den, nrm.d_mean, nrm.d_den,
                        nrm.r_mean, nrm.r_den, nrm.ret_den)
    eng.set_net("t1", [w * 0.5 for w in st.q_targ[1]])       # a target that differs from q1
    s, a, *_ = _rows(n, ocfg.S, ocfg.A, 2)
    for k, net, params in ((0, "q0", st.q[0]), (1, "q1", st.q[1]), (3, "t1", [w * 0.5 for w in st.q_targ[1]])):
        f = eng.critic_forward(net, s, a).cpu().numpy()
        v = eng.critic_forward(net, s, a, value=True).cpu().numpy()
        assert f.shape == (n, 1) and v.shape == (n,)
        rf = O.critic_forward([x.astype(np.float64) for x in params], ocfg, nrm, s, a)
        rv = O.critic_forward([x.astype(np.float64) for x in params], ocfg, nrm, s, a, value=True)
        assert relerr(f, rf) < 2e-5 and relerr(v, rv) < 2e-5, (net, relerr(f, rf), relerr(v, rv))
    eng.close()


@pytest.mark.parametrize("n,dclip,rclip", [(1, 0.0, 0.0), (300, 0.0, 0.0), (5000, 0.05, 0.3)])
def test_model_forward(gpu_available, n, dclip, rclip):
    eng, ocfg, st, buf, nrm, _ = make_pair(act="relu", B=64, seed=45, use_expert=True, normalizers="random")
    nrm.r_mean, nrm.r_den = np.float32(0.3), np.float32(1.7)
    eng.set_normalizers(nrm.s_mean, nrm.s_den, nrm.a_mean, nrm.a_den, nrm.d_mean, nrm.d_den,
                        nrm.r_mean, nrm.r_den, nrm.ret_den)
    s, a, *_ = _rows(n, ocfg.S, ocfg.A, 3)
    for k in range(2):
        pred, sp, r = [t.cpu().numpy() for t in eng.model_forward(k, s, a, dclip, rclip)]
        rp, rsp, rr = O.model_forward(st, ocfg, nrm, k, s, a, dclip, rclip)
        assert relerr(pred, rp) < 2e-5 and relerr(sp, rsp) < 2e-5 and relerr(r, rr) < 2e-5
        if dclip:
            assert np.max(np.abs(pred[:, :-1])) <= dclip
    eng.close()


@pytest.mark.parametrize("n,dclip,rclip", [(1, 0.0, 0.0), (200, 0.0, 0.0), (9000, 0.5, 1.0)])
def test_model_loss(gpu_available, n, dclip, rclip):
    eng, ocfg, st, buf, nrm, _ = make_pair(act="relu", B=64, seed=47, use_expert=True, normalizers="random")
    s, a, sp, r = _rows(n, ocfg.S, ocfg.A, 4)
    for k in range(2):
        got = eng.model_loss(k, s, sp, a, r, dclip, rclip)
        ref = O.model_loss(st, ocfg, nrm, k, s, sp, a, r, dclip, rclip)
        assert abs(got - ref) <= 1e-5 * abs(ref), (k, got, ref)
    eng.close()


def test_reference_objects_call_the_device(gpu_available):
    """The reference-named objects (bound to an engine as an algorithm binds them) return what
    the reference's methods return: shapes (incl. the one-row squeeze) and values."""
    from sac_eo.actors import init_actor
    from sac_eo.common.train_parser import create_train_parser, gather_inputs
    from sac_eo.critics import init_critics
    from sac_eo.envs import init_env
    from sac_eo.models import init_world_models
    eng, ocfg, st, buf, nrm, _ = make_pair(act="tanh", B=64, seed=49, use_expert=True)
    env = init_env("gym", "HalfCheetah-v3")
    k = gather_inputs(create_train_parser().parse_args(["--actor_layers", "256", "256", "--critic_layers", "256", "256",
                                                         "--actor_activations", "tanh", "--critic_activations",
                                                         "tanh", "--model_activations", "relu"]))
    actor = init_actor(env, **dict(k["actor_kwargs"], actor_weights=None, actor_squash=True))
    _, q_targets, q_critics = init_critics(env, **dict(k["critic_kwargs"], critic_weights=None))
    models = init_world_models(env, **dict(k["model_kwargs"], model_weights=None, reward_weights=None),
                               model_setup_kwargs=k["model_setup_kwargs"])
    actor.set_weights(st.actor + [st.logstd])
    actor._bind(eng, "actor")
    q_critics[0].set_weights(st.q[0])
    q_critics[0]._bind(eng, "q0")
    q_targets[1].set_weights(st.q_targ[1])
    q_targets[1]._bind(eng, "t1")
    models[1].set_weights(st.models[1])
    models[1]._bind(eng, "m1")
    s, a, sp, r = _rows(5, ocfg.S, ocfg.A, 5)
    eng.rng_set_state(np.random.RandomState(3).get_state())
    rs = np.random.RandomState(3)
    pi, nlp = actor.evaluate(s)
    rpi, rnlp = O.actor_evaluate(st, ocfg, nrm, s, rs)
    assert pi.shape == (5, 6) and nlp.shape == (5,) and relerr(pi, rpi) < 2e-5 and relerr(nlp, rnlp) < 2e-5
    pi1, nlp1 = actor.evaluate(s[:1])                      # one row: squeezed like the reference
    assert pi1.shape == (6,) and np.ndim(nlp1) == 0 and np.asarray(pi1.numpy()).shape == (6,)
    q = q_critics[0]._forward(s, a)
    v = q_targets[1].value(s, a)
    assert q.shape == (5, 1) and v.shape == (5,)
    assert relerr(q, O.critic_forward([x.astype(np.float64) for x in st.q[0]], ocfg, nrm, s, a)) < 2e-5
    assert relerr(v, O.critic_forward([x.astype(np.float64) for x in st.q_targ[1]], ocfg, nrm, s, a, True)) < 2e-5
    m = models[1]
    _, rsp, rr = O.model_forward(st, ocfg, nrm, 1, s, a)
    assert relerr(m.sample(s, a), rsp) < 2e-5
    dn, rn = m._forward(s, a)
    assert dn.shape == (5, ocfg.S) and rn.shape == (5,)
    m.reset(s)
    s1, r1, d1, _ = m.step(a)
    assert relerr(s1, rsp) < 2e-5 and relerr(r1, rr) < 2e-5 and not np.any(d1)
    loss = m.get_loss(s, sp, a, r)
    assert abs(loss - O.model_loss(st, ocfg, nrm, 1, s, sp, a, r)) <= 1e-5 * abs(loss)
    eng.close()
