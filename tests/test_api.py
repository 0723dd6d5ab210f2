"""Host API mirror on CPU: the reference's construction functions, weight-list layouts,
normaliser update rule, synthetic env and the train-flag parser (no GPU needed)."""
import numpy as np
import pytest

from sac_eo.actors import init_actor
from sac_eo.common.normalizer import RunningNormalizer, discounted_sum
from sac_eo.common.train_parser import create_train_parser, gather_inputs
from sac_eo.critics import init_critics
from sac_eo.envs import init_env
from sac_eo.models import init_world_models


def _kwargs(argv=()):
    args = create_train_parser().parse_args(list(argv))
    return gather_inputs(args)


def test_actor_weight_layout_matches_reference():
    env = init_env("gym", "HalfCheetah-v3")
    ak = _kwargs(["--actor_layers", "256", "256"])["actor_kwargs"]
    actor = init_actor(env, **dict(ak, actor_weights=None, actor_squash=True))
    w = actor.get_weights()
    shapes = [x.shape for x in w]
    # [W0(in,out), b0, W1, b1, W2, b2] + logstd (1, A)  (pinned by the reference's logs)
    assert shapes == [(17, 256), (256,), (256, 256), (256,), (256, 6), (6,), (1, 6)]
    assert np.all(w[-1] == 0) and np.all(w[1] == 0)
    # orthogonal init with gain: hidden sqrt(2), final actor_gain (0.01)
    q = w[2] / np.sqrt(2)
    assert np.allclose(q.T @ q, np.eye(256), atol=1e-4)
    assert np.isclose(np.linalg.svd(w[4], compute_uv=False).max(), 0.01, rtol=1e-4)
    # actor_squash False: the reference's plain GaussianActor (an imported expert, inference only)
    from sac_eo.actors import GaussianActor, SquashedGaussianActor
    g = init_actor(env, **dict(ak, actor_weights=w, actor_squash=False))
    assert type(g) is GaussianActor and not g.squash and isinstance(actor, SquashedGaussianActor)
    assert all(np.array_equal(a, b) for a, b in zip(g.get_weights(), w))
    # --actor_output_norm: the reference's squashed sample / evaluate never apply it
    # (continuous_actors.py:270-379), so the squashed actor accepts and ignores it
    # (an init_actor keyword, init_actor.py:10; the reference parser has no flag for it)
    sq = init_actor(env, **dict(ak, actor_weights=w, actor_squash=True, actor_output_norm=True))
    assert sq.output_norm and isinstance(sq, SquashedGaussianActor)


def test_critics_and_models_construction():
    env = init_env("gym", "Walker2d-v3")
    k = _kwargs(["--critic_layers", "256", "256"])
    critics, q_targets, q_critics = init_critics(env, **dict(k["critic_kwargs"], critic_weights=None))
    assert len(q_critics) == 2 and len(q_targets) == 2 and len(critics) == 1
    for t, q in zip(q_targets, q_critics):
        assert all(np.array_equal(a, b) for a, b in zip(t.get_weights(), q.get_weights()))
    assert [x.shape for x in q_critics[0].get_weights()] == [(23, 256), (256,), (256, 256), (256,), (256, 1), (1,)]
    models = init_world_models(env, **dict(k["model_kwargs"], model_weights=None, reward_weights=None),
                               model_setup_kwargs=k["model_setup_kwargs"])
    assert len(models) == 2
    assert [x.shape for x in models[0].get_weights()][0::2] == [(23, 512), (512, 512), (512, 18)]


def test_running_normalizer_matches_batch_statistics():
    """normalizer.py update(): after several batches mean/var equal the pooled sample stats."""
    rs = np.random.RandomState(0)
    data = rs.normal(size=(300, 4)).astype(np.float32) * [1, 2, 3, 4] + [0, 1, -1, 5]
    n = RunningNormalizer(4)
    for chunk in np.array_split(data, [50, 120, 121, 299]):
        n.update(chunk)
    assert np.allclose(n.mean, data.mean(axis=0), atol=1e-4)
    assert np.allclose(n.var, data.var(axis=0, ddof=1), rtol=1e-3)
    assert np.allclose(discounted_sum([1, 1, 1], 0.5), [1.75, 1.5, 1.0])


def test_synthetic_env_gym_api():
    env = init_env("gym", "Humanoid-v3")
    assert env.observation_space.shape == (376,) and env.action_space.shape == (17,)
    assert np.all(env.action_space.low == -1) and np.all(env.action_space.high == 1)
    env.seed(3)
    s0 = env.reset()
    s1, r, d, info = env.step(np.zeros(17))
    env.seed(3)
    assert np.array_equal(env.reset(), s0) and np.array_equal(env.step(np.zeros(17))[0], s1)
    st = np.random.get_state()
    env.step(np.ones(17))
    assert np.array_equal(np.random.get_state()[1], st[1])    # env never touches the global stream
    with pytest.raises(ValueError):
        init_env("gym", "NoSuchEnv-v0")


def test_train_parser_reference_defaults():
    k = _kwargs([])
    assert k["alg_kwargs"]["alg_type"] == "sac_imit"
    assert k["alg_kwargs"]["sac_batch_size"] == 256 and k["alg_kwargs"]["soft_tau"] == 5e-3
    assert k["alg_kwargs"]["q_crit_lr"] == 3e-4 and k["alg_kwargs"]["mbpo_actor_lr"] == 1e-4
    assert k["model_kwargs"]["model_layers"] == [512, 512]
    assert k["alg_kwargs"]["model_batch_shuffle"] is True
    assert _kwargs(["--no_model_batch_shuffle"])["alg_kwargs"]["model_batch_shuffle"] is False
