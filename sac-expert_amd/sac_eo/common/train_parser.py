"""Command-line flags of ``python -m sac_eo.train``.

Same flag names, types, defaults and kwargs groups as the reference parser
(sac_eo/common/train_parser.py:8-439) so existing command lines and logged
``param`` dicts carry over.  Flags the reference accepts but never reads
("Dead flags") are accepted and ignored here too.  One addition
in the setup group: ``--gpus`` (learners are placed one per GPU) and ``--serial_runs`` (run the
``--runs`` of one process one after another instead of as lock-step packed seeds).
"""
import argparse

F, I, S = float, int, str
T = "store_true"
SAME = "same"   # a second kwargs group for a flag defined earlier (no new parser argument)

# (group, flag, type_or_action, default, extra).  The rows are in the reference's order within each
# kwargs group (all_kwargs is the logged ``param`` layout, pinned by tests/golden/ref_fixtures.json);
# group None = a parser flag in no kwargs group (--alg_seed)
_FLAGS = [
    # setup
    ("setup", "runs", I, 1, {}), ("setup", "runs_start", I, 0, {}), ("setup", "cores", I, None, {}),
    ("setup", "seed", I, 0, {}), ("setup", "setup_seed", I, None, {}), ("setup", "sim_seed", I, None, {}),
    ("setup", "eval_seed", I, None, {}), ("setup", "expert_seed", I, None, {}), (None, "alg_seed", I, None, {}),
    ("setup", "save_path", S, "./logs", {}), ("setup", "save_file", S, None, {}),
    ("setup", "import_path", S, "./logs", {}), ("setup", "import_file", S, None, {}),
    ("setup", "import_idx", I, None, {}), ("setup", "import_all", T, False, {}),
    ("setup", "expert_file", S, None, {}), ("setup", "expert_path", S, "./experts", {}),
    ("setup", "gpus", I, None, {}), ("setup", "serial_runs", T, False, {}),
    # environment
    ("env", "env_type", S, "gym", {}), ("env", "env_name", S, "Pendulum-v1", {}), ("env", "task_name", S, None, {}),
    # actor
    ("actor", "actor_layers", I, [64, 64], {"nargs": "+"}), ("actor", "actor_activations", S, ["tanh"], {"nargs": "+"}),
    ("actor", "actor_gain", F, 0.01, {}), ("actor", "actor_std_mult", F, 1.0, {}),
    ("actor", "actor_init_type", S, "orthogonal", {}), ("actor", "actor_layer_norm", T, False, {}),
    ("actor", "actor_per_state_std", T, False, {}), ("actor", "actor_squash", T, False, {}),
    # critic
    ("critic", "critic_layers", I, [64, 64], {"nargs": "+"}), ("critic", "critic_activations", S, ["tanh"], {"nargs": "+"}),
    ("critic", "critic_gain", F, 1.0, {}), ("critic", "critic_ensemble", T, False, {}),
    ("critic", "num_models", I, 2, {}), ("critic", "critic_init_type", S, "orthogonal", {}),
    ("critic", "critic_layer_norm", T, False, {}),
    # model
    ("model", "gaussian_model", T, False, {}), ("model", "num_models", SAME, None, {}),
    ("model", "model_layers", I, [512, 512], {"nargs": "+"}), ("model", "model_activations", S, ["relu"], {"nargs": "+"}),
    ("model", "model_gain", F, 0.01, {}), ("model", "model_std_mult", F, 1.0, {}),
    ("model", "reward_layers", I, [512, 512], {"nargs": "+"}), ("model", "reward_activations", S, ["relu"], {"nargs": "+"}),
    ("model", "reward_gain", F, 0.01, {}),
    # model setup
    ("model_setup", "separate_reward_nn", T, False, {}), ("model_setup", "reward_loss_coef", F, 1.0, {}),
    ("model_setup", "scale_model_loss", T, False, {}), ("model_setup", "delta_clip_loss", F, None, {}),
    ("model_setup", "reward_clip_loss", F, None, {}), ("model_setup", "delta_clip_pred", F, None, {}),
    ("model_setup", "reward_clip_pred", F, None, {}),
    # buffers
    ("alg", "gamma", F, 0.995, {}), ("alg", "lam", F, 0.97, {}), ("alg", "env_buffer_size", F, None, {}),
    ("alg", "sim_buffer_size", F, None, {}), ("alg", "model_buffer_size", F, 1e5, {}),
    ("alg", "expert_buffer_size", F, 20, {}),
    # training
    ("alg", "save_path", SAME, None, {}), ("alg", "checkpoint_file", S, "TEMPLOG", {}), ("alg", "save_freq", F, None, {}),
    ("alg", "eval_freq", F, None, {}), ("alg", "eval_num_traj", I, 5, {}),
    ("alg", "alg_type", S, "sac_imit", {}), ("alg", "mf_algo", S, "trpo", {}),
    ("alg", "total_timesteps", F, 5e5, {}), ("alg", "env_horizon", I, 1000, {}),
    ("alg", "env_batch_type", S, "steps", {"choices": ["steps", "traj"]}),
    ("alg", "env_batch_size_init", I, 5000, {}), ("alg", "env_batch_size", I, 3000, {}),
    ("alg", "s_noise_std", F, 0.0, {}), ("alg", "s_noise_type", S, "all", {"choices": ["all", "next"]}),
    ("alg", "sim_horizon", I, 5, {}), ("alg", "sim_batch_type", S, "steps", {"choices": ["steps", "traj"]}),
    ("alg", "sim_batch_size", I, 10000, {}), ("alg", "exp_batch_type", S, "steps", {"choices": ["steps", "traj"]}),
    # model update
    ("alg", "model_lr", F, 1e-3, {}), ("alg", "model_num_epochs", I, 10, {}), ("alg", "model_batch_size", I, 200, {}),
    # model-update batch shuffling is a negative flag in the reference (--no_model_batch_shuffle)
    ("alg", "model_batch_shuffle", "store_false_alias:no_model_batch_shuffle", True, {}),
    ("alg", "model_max_updates", F, 1e5, {}), ("alg", "model_max_grad_norm", F, None, {}),
    ("alg", "model_holdout_ratio", F, 0.0, {}), ("alg", "model_holdout_epochs", I, 5, {}),
    ("alg", "reset_model_optimizer", T, False, {}),
    # on-policy actor-critic (kept for the param dict)
    ("alg", "critic_lr", F, 3e-4, {}), ("alg", "critic_update_it", I, 10, {}), ("alg", "critic_nminibatch", I, 32, {}),
    ("alg", "num_mf_updates", I, 25, {}),
    # SAC-EO expert regulariser
    ("alg", "epsilon", F, 1e-3, {}), ("alg", "scale_epsilon_by_true_MSE", T, False, {}),
    ("alg", "scale_max_disc", T, False, {}), ("alg", "scale_median_disc", T, False, {}),
    ("alg", "scale_total_disc", T, False, {}), ("alg", "use_expert_actions", T, False, {}),
    ("alg", "min_mult", T, False, {}), ("alg", "exp_mult", T, False, {}), ("alg", "mult_coeff", F, 1.0, {}),
    ("alg", "init_from_expert", T, False, {}), ("alg", "max_exp_state_ratio", F, 0.25, {}),
    # SAC / MBPO
    ("alg", "init_temperature", F, 1e-1, {}), ("alg", "q_crit_lr", F, 3e-4, {}), ("alg", "mbpo_actor_lr", F, 1e-4, {}),
    ("alg", "mbpo_alpha_lr", F, 1e-4, {}), ("alg", "mbpo_E", I, 1000, {}), ("alg", "mbpo_G", I, 3, {}),
    ("alg", "mbpo_M", I, 400, {}), ("alg", "sac_batch_size", I, 256, {}), ("alg", "expert_batch_size", I, None, {}),
    ("alg", "soft_tau", F, 5e-3, {}), ("alg", "target_update_int", I, 1, {}), ("alg", "real_step_mod", I, 3, {}),
    ("alg", "random_act", T, False, {}), ("alg", "update_normalizers", T, False, {}),
    ("alg", "only_model_normalizer", T, False, {}), ("alg", "adaptive_model_horizon", T, False, {}),
    ("alg", "modelhorx", F, 1, {}), ("alg", "modelhory", F, 15, {}), ("alg", "modelhora", F, 20, {}),
    ("alg", "modelhorb", F, 100, {}),
    # model-free on-policy updates (mf_update_kwargs)
    ("mf", "adv_center", "store_false_alias:no_adv_center", True, {}),
    ("mf", "adv_scale", "store_false_alias:no_adv_scale", True, {}),
    ("mf", "ent_reg", T, False, {}), ("mf", "alpha_lr", F, 3e-4, {}),
    ("mf", "delta_trpo", F, 0.02, {}), ("mf", "cg_it", I, 20, {}), ("mf", "trust_sub", I, 1, {}),
    ("mf", "trust_damp", F, 0.01, {}), ("mf", "kl_maxfactor", F, 1.5, {}),
    ("mf", "actor_update_it", I, 10, {}), ("mf", "actor_nminibatch", I, 32, {}), ("mf", "actor_lr", F, 3e-4, {}),
    ("mf", "eps_ppo", F, 0.2, {}), ("mf", "max_grad_norm", F, 0.5, {}),
    ("mf", "adaptlr", "store_false_alias:no_adaptlr", True, {}), ("mf", "adapt_factor", F, 0.03, {}),
    ("mf", "adapt_minthresh", F, 0.0, {}), ("mf", "adapt_maxthresh", F, 1.0, {}),
]

_GROUP_NAMES = {"setup": "setup_kwargs", "env": "env_kwargs", "actor": "actor_kwargs", "critic": "critic_kwargs",
                "model": "model_kwargs", "model_setup": "model_setup_kwargs", "alg": "alg_kwargs",
                "mf": "mf_update_kwargs"}

all_kwargs = {v: [] for v in _GROUP_NAMES.values()}
for grp, name, _t, _d, extra in _FLAGS:
    if grp is None or name in ("gpus", "serial_runs"):
        continue   # parser-only flags, and the local additions
    all_kwargs[_GROUP_NAMES[grp]].append(name)


def create_train_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="MI355X SAC / SAC-EO training (noc-lab/sac-expert compatible flags)")
    for _grp, name, typ, default, extra in _FLAGS:
        kw = {k: v for k, v in extra.items() if k in ("nargs", "choices")}
        if typ == SAME:
            continue
        if typ == T:
            p.add_argument("--" + name, action="store_true")
        elif isinstance(typ, str) and typ.startswith("store_false_alias:"):
            p.add_argument("--" + typ.split(":", 1)[1], dest=name, default=default, action="store_false")
        else:
            p.add_argument("--" + name, type=typ, default=default, **kw)
    return p


def gather_inputs(args) -> dict:
    """train_utils.py:6-18: argparse namespace -> grouped kwargs dicts."""
    a = vars(args)
    return {grp: {k: a[k] for k in names} for grp, names in all_kwargs.items()}
