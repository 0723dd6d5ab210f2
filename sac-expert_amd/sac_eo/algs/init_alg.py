"""init_alg (reference ``sac_eo/algs/init_alg.py:9-34``)."""
from .SAC import SAC
from .SAC_expert import SAC_exp


def init_alg(idx, env, env_eval, env_expert, actor, critics, q_targets, q_critics, models, alg_kwargs,
             mf_update_kwargs, expert, init_expert_rms_stats):
    alg_type = alg_kwargs["alg_type"]
    if alg_type == "sac":
        return SAC(idx, env, env_eval, actor, critics, q_targets, q_critics, models, alg_kwargs, mf_update_kwargs)
    if alg_type == "sac_imit":
        return SAC_exp(idx, env, env_eval, env_expert, actor, expert, init_expert_rms_stats, critics, q_targets,
                       q_critics, models, alg_kwargs, mf_update_kwargs)
    if alg_type in ("mbrl", "bc"):
        raise NotImplementedError(f"alg_type {alg_type!r} is outside the SAC / SAC-EO path built here")
    raise ValueError("invalid alg_type")
