"""The drop-in TRAINING LOOP against an oracle-driven restatement of it.

``SAC_exp.train`` (sac_eo/algs/SAC_expert.py:685-824) and ``SAC.train`` (sac_eo/algs/SAC.py:254-385)
run on the device (``sac_eo.algs``: behaviour actions, replay appends, gradient steps, model
fits and expert diagnostics through libsacx) and on the CPU (``oracle/sac_loop.py``: the same
loop over ``sac_oracle`` in fp64), on the same synthetic environments, initial weights, global
NumPy stream and expert-permutation Generator.  Compared:

* every update's Q1 / Q2 / policy / alpha loss (relative to the trajectory's scale),
* the global NumPy stream (MT19937 key, position, cached gauss) at every episode boundary,
  bit for bit -- it carries the sampler, the actor noise, the model-fit shuffles, the expert
  batch draw and the counterfactual actions of the diagnostics in the reference's order,
* SAC-EO's per-episode expert MSE diagnostics and last model-fit loss,
* with ``--update_normalizers`` (per-trajectory merge during the initial collection, per-episode
  merge of new_traj, :740-746) and ``--only_model_normalizer`` (the world models on their own
  normaliser, :53-54 / :139-144 / :646-650), whose normaliser statistics must also agree.
"""
import numpy as np
import pytest

import sac_oracle as O
from sac_loop import LoopOracle

pytestmark = pytest.mark.gpu

LOSS_TOL = 1e-4      # north_star: Q-loss trajectory within 1e-4 relative
# the loop shapes: SMALL runs every flag variant fast; BENCH is the metric's configuration
# (256x2 nets, B = 256, 512x2 world models, model minibatch 200, 100-step episodes)
SMALL = dict(hidden=64, B=64, model_hidden=64, model_batch=50, epochs=2, ep_len=40, init=200, episodes=3)
BENCH = dict(hidden=256, B=256, model_hidden=512, model_batch=200, epochs=3, ep_len=100, init=400, episodes=3)


def _build(alg, flags, seed=7, shape=SMALL, act="relu"):
    """The construction sequence of sac_eo/train.py:28-59 with short synthetic episodes."""
    from sac_eo.actors import init_actor
    from sac_eo.algs import init_alg
    from sac_eo.common.seeding import derive_seeds, init_seeds
    from sac_eo.common.train_parser import create_train_parser, gather_inputs
    from sac_eo.critics import init_critics
    from sac_eo.envs.synthetic import SyntheticEnv
    from sac_eo.models import init_world_models
    ep_len = shape["ep_len"]
    total = shape["init"] + shape["episodes"] * ep_len
    h, mh = str(shape["hidden"]), str(shape["model_hidden"])
    argv = ["--alg_type", alg, "--env_name", "HalfCheetah-v3", "--actor_layers", h, h,
            "--critic_layers", h, h, "--actor_activations", act, "--critic_activations", act,
            "--model_layers", mh, mh, "--total_timesteps", str(total), "--env_batch_size_init", str(shape["init"]),
            "--env_horizon", "1000", "--sac_batch_size", str(shape["B"]), "--model_batch_size",
            str(shape["model_batch"]), "--model_num_epochs", str(shape["epochs"]), "--seed", str(seed)] + flags
    d = gather_inputs(create_train_parser().parse_args(argv))
    d["actor_kwargs"]["actor_squash"] = True
    sd = derive_seeds(seed, 1, 0)
    ak = dict(d["alg_kwargs"], alg_seed=int(sd["algorithm"][0]), save_path="/tmp/sacx_loop_test")
    init_seeds(int(sd["setup"][0]))
    envs = [SyntheticEnv("HalfCheetah-v3", max_episode_steps=ep_len) for _ in range(3)]
    actor = init_actor(envs[0], **dict(d["actor_kwargs"], actor_weights=None))
    expert = init_actor(envs[0], **dict(d["actor_kwargs"], actor_weights=None))
    critics, q_targets, q_critics = init_critics(envs[0], **dict(d["critic_kwargs"], critic_weights=None))
    models = init_world_models(envs[0], **dict(d["model_kwargs"], model_weights=None, reward_weights=None),
                               model_setup_kwargs=d["model_setup_kwargs"])
    init_seeds(int(sd["eval"][0]), envs[1])
    init_seeds(int(sd["sim"][0]), envs[0])
    init_seeds(int(sd["expert"][0]), envs[2])
    alg_obj = init_alg(0, envs[0], envs[1], envs[2], actor, critics, q_targets, q_critics, models, ak,
                       d["mf_update_kwargs"], expert, None)
    # what the oracle starts from: the bound weights, the global stream, fresh env copies
    oenvs = [SyntheticEnv("HalfCheetah-v3", max_episode_steps=ep_len) for _ in range(3)]
    oenvs[0].seed(int(sd["sim"][0]))
    oenvs[2].seed(int(sd["expert"][0]))
    return alg_obj, d, ak, total, oenvs, np.random.get_state()


def _oracle_state(alg_obj, ocfg):
    aw = alg_obj.actor.get_weights()
    q = [c.get_weights() for c in alg_obj.q_critics]
    qt = [t.get_weights() for t in alg_obj.q_targets]
    alpha = np.asarray(np.float32(np.log(ocfg.init_temperature)), np.float32)     # SAC_expert.py:106
    st = O.SACState(aw[:-1], aw[-1], q, qt, alpha, O.AdamState.zeros_like(aw),
                    [O.AdamState.zeros_like(n) for n in q], O.AdamState.zeros_like([alpha]))
    if alg_obj.use_expert:
        ws = [m.get_weights() for m in alg_obj.models]
        if ocfg.gaussian_model:            # GaussianModel.get_weights: the net's weights + [logstd]
            st.models = [w[:-1] for w in ws]
            st.model_logstd = [w[-1] for w in ws]
        else:
            st.models = ws
        if ocfg.separate_reward_nn:
            st.reward_nets = [m.get_reward_weights() for m in alg_obj.models]
        st.opt_model = O.AdamState.zeros_like(st.model_all_vars())
    return st.astype(np.float64)


def _series_err(dev, ref):
    return float(np.max(np.abs(dev - ref)) / max(np.max(np.abs(ref)), 1e-30))


def _rel_drift(a, b):
    """Largest elementwise relative difference (per episode: the diagnostics are not a series)."""
    return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1e-30))) if b.size else 0.0


def _same_stream(a, b):
    return np.array_equal(a[1], b[1]) and a[2] == b[2] and a[3] == b[3] and a[4] == b[4]


def _fresh_envs(shape):
    from sac_eo.common.seeding import derive_seeds
    from sac_eo.envs.synthetic import SyntheticEnv
    sd = derive_seeds(7, 1, 0)
    e = [SyntheticEnv("HalfCheetah-v3", max_episode_steps=shape["ep_len"]) for _ in range(3)]
    e[0].seed(int(sd["sim"][0]))
    e[2].seed(int(sd["expert"][0]))
    return e


def _run(alg, flags, shape=SMALL, act="relu", fp32_envelope=False):
    """The device loop and the fp64 oracle loop from the same start; returns everything compared."""
    alg_obj, d, ak, total, oenvs, rs_state = _build(alg, flags, shape=shape, act=act)
    S, A = alg_obj.s_dim, alg_obj.a_dim
    mk, msk = d["model_kwargs"], d["model_setup_kwargs"]
    # the parsed layer lists (a flag given again in `flags` replaces the shape's: nargs='+')
    ocfg = O.Config(S=S, A=A, hidden=tuple(d["actor_kwargs"]["actor_layers"]), act=act, B=shape["B"], gamma=ak["gamma"],
                    tau=ak["soft_tau"], lr_q=ak["q_crit_lr"], lr_pi=ak["mbpo_actor_lr"], lr_alpha=ak["mbpo_alpha_lr"],
                    init_temperature=ak["init_temperature"], epsilon=ak["epsilon"],
                    model_hidden=tuple(mk["model_layers"]), num_models=int(mk["num_models"]),
                    layer_norm=bool(d["actor_kwargs"].get("actor_layer_norm", False)),
                    model_act="relu", lr_model=ak["model_lr"], reward_loss_coef=msk["reward_loss_coef"],
                    gaussian_model=bool(mk["gaussian_model"]),
                    scale_model_loss=bool(msk["scale_model_loss"]) and bool(mk["gaussian_model"]),
                    separate_reward_nn=bool(msk["separate_reward_nn"]), reward_hidden=tuple(mk["reward_layers"]),
                    reward_act=mk["reward_activations"][0],
                    critic_hidden=tuple(d["critic_kwargs"]["critic_layers"]))
    st = _oracle_state(alg_obj, ocfg)
    # the fp32 envelope starts from the SAME initial state: sac_update / model_fit_step advance
    # the state they are given in place, so it is copied before the fp64 run trains st
    st32 = st.astype(np.float32) if fp32_envelope else None
    expert = None
    if alg == "sac_imit":
        ex = alg_obj.expert.get_weights()
        expert = ([np.asarray(w, np.float64) for w in ex[:-1]], np.asarray(ex[-1], np.float64))
    # the device loop, with the global stream recorded at every episode boundary
    dev_rng = []
    hook = alg_obj._episode_normalizer_update

    def rec(episode):
        dev_rng.append(alg_obj.engine.rng_get_state())
        return hook(episode)
    alg_obj._episode_normalizer_update = rec
    name = alg_obj.train(total, d)
    dev_rng.append(alg_obj.engine.rng_get_state())
    n_upd = alg_obj.engine.ctl()["step_seq"]
    dev = alg_obj.engine.stats(n_upd)
    ok = dict(ak, num_models=d["model_kwargs"]["num_models"])
    orc = LoopOracle(alg, ocfg, st, oenvs[0], oenvs[2], expert, ok, rs_state, ak["alg_seed"],
                     max_episode_steps=1000).train(total)
    ref = np.array([[u["q1_loss"], u["q2_loss"], u["p_loss"], u["alpha_loss"]] for u in orc.update_stats])
    env32 = None
    if fp32_envelope:
        # the drift a faithful fp32 execution has: the same loop in fp32 against the fp64 one
        e32 = _fresh_envs(shape)
        ex32 = None if expert is None else ([w.astype(np.float32) for w in expert[0]], expert[1].astype(np.float32))
        o32 = LoopOracle(alg, ocfg, st32, e32[0], e32[2], ex32, ok, rs_state, ak["alg_seed"],
                         max_episode_steps=1000).train(total)
        r32 = np.array([[u["q1_loss"], u["q2_loss"], u["p_loss"], u["alpha_loss"]] for u in o32.update_stats])
        env32 = [_series_err(r32[:, c], ref[:, c]) for c in range(4)]
        if alg == "sac_imit":
            # the same drift for the per-episode diagnostics (model MSEs) and last fit losses
            env32.append(_rel_drift(np.array(o32.diag), np.array(orc.diag)))
            env32.append(_rel_drift(np.array(o32.fit_last), np.array(orc.fit_last)))
    return alg_obj, ak, name, dev, dev_rng, orc, ref, env32


def _check_stream_and_diag(alg, flags, alg_obj, ak, name, dev_rng, orc, tol=LOSS_TOL):
    """``tol``: the bar for the per-episode expert diagnostics and last model-fit losses (relative to
    each value): 1e-4 at the small shapes, 1e-3 at the bench shapes (three episodes of 300 updates
    and 3 x 6 model-fit epochs of 512-wide nets between the diagnostics)."""
    assert len(dev_rng) == len(orc.episode_rng)
    for i, (a, b) in enumerate(zip(dev_rng, orc.episode_rng)):
        assert _same_stream(a, b), f"global stream differs at episode boundary {i}"
    if "--update_normalizers" in flags:
        for which in ("normalizer", "model_normalizer"):
            mine, theirs = getattr(alg_obj, which), getattr(orc, which)
            for kk in ("s_rms", "a_rms", "r_rms", "delta_rms", "ret_rms"):
                a, b = getattr(mine, kk), getattr(theirs, kk)
                assert a.t_last == b.t_last, (which, kk)
                np.testing.assert_allclose(np.asarray(a.mean, np.float64), np.asarray(b.mean, np.float64),
                                           rtol=1e-5, atol=1e-6, err_msg=f"{which}.{kk}")
                np.testing.assert_allclose(np.asarray(a.var, np.float64), np.asarray(b.var, np.float64),
                                           rtol=1e-4, atol=1e-6, err_msg=f"{which}.{kk}")
    if alg == "sac_imit":
        from sac_eo.common.logger import load_log
        import os
        log = load_log(os.path.join(ak["save_path"], name))
        dd = np.asarray(log["train"]["model_MSE_on_expert_data"], np.float64)
        dc = np.asarray(log["train"]["model_MSE_on_expert_counterfactual_action"], np.float64)
        od = np.array(orc.diag)
        assert len(dd) == len(od)
        tol_d = tol_f = tol
        print(f"diagnostics: rel err {_rel_drift(np.stack([dd, dc], 1), od[:, :2]):.2e} (tol {tol_d:.2e}), "
              f"fit loss {_rel_drift(np.asarray(log['train']['model_loss_last'], np.float64), np.array(orc.fit_last)):.2e} "
              f"(tol {tol_f:.2e})")
        np.testing.assert_allclose(dd, od[:, 0], rtol=tol_d)
        np.testing.assert_allclose(dc, od[:, 1], rtol=tol_d)
        ml = np.asarray(log["train"]["model_loss_last"], np.float64)
        assert len(ml) == len(orc.fit_last)
        np.testing.assert_allclose(ml, np.array(orc.fit_last), rtol=tol_f)   # sum over the models, last fit step
        os.remove(os.path.join(ak["save_path"], name))


@pytest.mark.parametrize("alg,flags", [
    ("sac_imit", []),
    ("sac_imit", ["--update_normalizers"]),
    ("sac_imit", ["--update_normalizers", "--only_model_normalizer"]),
    ("sac_imit", ["--model_holdout_ratio", "0.2"]),
    ("sac_imit", ["--update_normalizers", "--s_noise_std", "0.3"]),
    ("sac_imit", ["--update_normalizers", "--s_noise_std", "0.3", "--s_noise_type", "next"]),
    ("sac_imit", ["--gaussian_model", "--model_std_mult", "0.5"]),
    ("sac_imit", ["--gaussian_model", "--scale_model_loss", "--separate_reward_nn", "--reward_layers", "48", "32",
                  "--reward_activations", "tanh"]),
    ("sac_imit", ["--separate_reward_nn", "--reward_layers", "64", "64", "--num_models", "1"]),
    ("sac", []),
    ("sac", ["--update_normalizers"]),
    ("sac", ["--update_normalizers", "--s_noise_std", "0.5"]),
    ("sac", ["--critic_layers", "96", "48"]),                 # critics wider / narrower than the actor
    ("sac_imit", ["--critic_layers", "40", "72"]),
    # round 6: nets of any depth (create_nn's layers list, nn_utils.py:100-138) and more world models
    ("sac", ["--actor_layers", "256", "256", "256"]),
    ("sac", ["--critic_layers", "400", "300", "200"]),
    ("sac_imit", ["--model_layers", "200", "200", "200"]),
    ("sac_imit", ["--actor_layers", "64"]),
    ("sac", ["--critic_layers", "96", "--actor_layers", "48", "80", "64", "32"]),
    ("sac_imit", ["--num_models", "3"]),
    ("sac_imit", ["--num_models", "4", "--gaussian_model", "--model_layers", "48", "64", "48"]),
    ("sac_imit", ["--separate_reward_nn", "--reward_layers", "48", "32", "40", "--model_layers", "64"]),
    ("sac", ["--actor_layer_norm", "--actor_layers", "64", "48", "64"]),
])
def test_train_loop_matches_oracle(gpu_available, alg, flags):
    alg_obj, ak, name, dev, dev_rng, orc, ref, _ = _run(alg, flags)
    assert dev.shape[0] == ref.shape[0], (dev.shape, ref.shape)
    errs = [_series_err(dev[:, c], ref[:, c]) for c in range(4)]
    print(f"{alg} {flags}: {dev.shape[0]} updates, errors q1 {errs[0]:.2e} q2 {errs[1]:.2e} p {errs[2]:.2e} "
          f"alpha {errs[3]:.2e}")
    _check_stream_and_diag(alg, flags, alg_obj, ak, name, dev_rng, orc)
    assert max(errs) < LOSS_TOL, errs            # all four series, alpha loss included
    alg_obj.engine.close()


@pytest.mark.parametrize("alg,act,flags", [
    ("sac_imit", "tanh", []),                       # the parser's default activation, 2 world models
    ("sac_imit", "relu", ["--num_models", "1"]),
    ("sac", "tanh", []),
    ("sac", "relu", []),
    ("sac", "relu", ["--critic_layers", "400", "300"]),       # --actor_layers 256 256 --critic_layers 400 300
])
def test_train_loop_bench_config(gpu_available, alg, act, flags):
    """The loops at the metric's shapes (256x2, B = 256, 512x2 models, minibatch 200, three
    100-step episodes after a 400-step collection): the global stream bit for bit at every episode
    boundary; every update's four losses within 1e-4 relative over the first 100 updates (north_star)
    and within 1e-3 over the whole run; the expert diagnostics and model-fit losses within 1e-3.

    The drift of a faithful fp32 execution (the same oracle loop in fp32 from the same start against
    the fp64 one) is printed beside the errors as a diagnostic, and must itself be small (< 1e-2):
    an envelope that wide would mean the two oracle loops do not run the same loop."""
    alg_obj, ak, name, dev, dev_rng, orc, ref, env32 = _run(alg, flags, shape=BENCH, act=act, fp32_envelope=True)
    assert dev.shape[0] == ref.shape[0] >= 200, (dev.shape, ref.shape)
    head = [_series_err(dev[:100, c], ref[:100, c]) for c in range(4)]
    full = [_series_err(dev[:, c], ref[:, c]) for c in range(4)]
    print(f"{alg} {act} {flags}: {dev.shape[0]} updates; first 100: {['%.2e' % e for e in head]}; "
          f"all: {['%.2e' % e for e in full]}; fp32 oracle drift {['%.2e' % e for e in env32]}")
    assert max(env32) < 1e-2, ("fp32 oracle loop diverges from the fp64 one: mis-specified envelope", env32)
    _check_stream_and_diag(alg, flags, alg_obj, ak, name, dev_rng, orc, tol=1e-3)
    assert max(head) < LOSS_TOL, head
    assert max(full) < 1e-3, full
    alg_obj.engine.close()
