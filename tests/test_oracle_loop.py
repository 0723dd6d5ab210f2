"""CPU checks of the loop oracle (oracle/sac_loop.py), the checker of tests/test_gpu_loop.py.

* Its global-stream consumption does not depend on float values: the fp64 and fp32 runs of
  the same loop leave the stream bit-identical at every episode boundary (so the device
  loop's stream can be held to bit-exactness whatever its rounding).
* Its RunningNormalizers restatement equals the product's host normaliser
  (sac_eo/common/normalizer.py) and scipy's lfilter discounted sum, bit for bit.
"""
import numpy as np
import pytest

import sac_oracle as O
from sac_loop import LoopOracle, RunningNorms, discounted_sum


def _loop(alg, dt, flags=()):
    from sac_eo.envs.synthetic import SyntheticEnv
    cfg = O.Config(S=17, A=6, hidden=(32, 32), act="relu", B=32, model_hidden=(32, 32))
    st = O.init_state(cfg, seed=3, with_models=alg == "sac_imit", bias_scale=0.05, actor_gain=0.5,
                      model_gain=0.3).astype(dt)
    ex = O.init_state(cfg, seed=4)
    envs = [SyntheticEnv("HalfCheetah-v3", max_episode_steps=25) for _ in range(2)]
    envs[0].seed(11)
    envs[1].seed(12)
    k = dict(gamma=0.99, epsilon=1e-3, env_batch_size_init=100, env_horizon=60, model_batch_size=40,
             model_num_epochs=1, num_models=2, expert_buffer_size=20, target_update_int=1, mbpo_G=3,
             real_step_mod=3, soft_tau=5e-3)
    for f in flags:
        k[f] = True
    rs = np.random.RandomState(5)
    return LoopOracle(alg, cfg, st, envs[0], envs[1], (ex.actor, ex.logstd), k, rs.get_state(), 9).train(100 + 50)


@pytest.mark.parametrize("alg,flags", [("sac_imit", ()), ("sac", ()),
                                       ("sac_imit", ("update_normalizers", "only_model_normalizer"))])
def test_stream_is_value_independent(alg, flags):
    a = _loop(alg, np.float64, flags)
    b = _loop(alg, np.float32, flags)
    assert len(a.episode_rng) == len(b.episode_rng) >= 3
    for x, y in zip(a.episode_rng, b.episode_rng):
        assert np.array_equal(x[1], y[1]) and x[2:] == y[2:]
    ra = np.array([[u["q1_loss"], u["p_loss"]] for u in a.update_stats])
    rb = np.array([[u["q1_loss"], u["p_loss"]] for u in b.update_stats])
    drift = np.max(np.abs(ra - rb), axis=0) / np.max(np.abs(ra), axis=0)
    print(f"{alg} {flags}: {len(ra)} updates, fp32-vs-fp64 loss drift {drift}")
    assert np.all(np.isfinite(ra)) and np.all(drift < 1e-2)


def test_normalizer_restatement_matches_host():
    from sac_eo.common.normalizer import RunningNormalizers, discounted_sum as host_ds
    import scipy.signal as sg
    rs = np.random.RandomState(0)
    mine, host = RunningNorms(5, 2, 0.99), RunningNormalizers(5, 2, 0.99)
    for n in (1, 7, 40, 3):
        s = rs.normal(size=(n, 5)).astype(np.float32) * 3
        a = rs.uniform(-1, 1, size=(n, 2)).astype(np.float32)
        r = rs.normal(size=n)                                  # float64, as new_traj holds it
        sp = s + rs.normal(size=(n, 5)).astype(np.float32)
        mine.update_rms(s, a, r, sp)
        host.update_rms(s, a, r, sp)
        ref = sg.lfilter([1], [1, -0.99], r[::-1], axis=0)[::-1]
        assert np.array_equal(discounted_sum(r, 0.99), ref) and np.array_equal(host_ds(r, 0.99), ref)
    for kk in ("s_rms", "a_rms", "r_rms", "delta_rms", "ret_rms"):
        x, y = getattr(mine, kk), getattr(host, kk)
        assert x.t_last == y.t_last
        assert np.array_equal(np.asarray(x.mean), np.asarray(y.mean)) and np.array_equal(np.asarray(x.var), np.asarray(y.var))
