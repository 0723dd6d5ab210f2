"""``python -m sac_eo.train`` (reference ``sac_eo/train.py``): same flags, seeds and
construction sequence, one learner per process.

Runs are spread over processes: under ``torch.distributed.run`` rank r trains run
``runs_start + r`` on its local GPU; otherwise the runs execute one after another on
the current GPU.  No data moves between learners (replicas)."""
import os
import sys
from datetime import datetime

import numpy as np

from .actors import init_actor
from .algs import init_alg
from .common.seeding import derive_seeds, init_seeds
from .common.train_parser import create_train_parser, gather_inputs
from .critics import init_critics
from .envs import init_env
from .models import init_world_models


def train(inputs_dict):
    """Training on one seed (reference train.py:33-100)."""
    sk = inputs_dict["setup_kwargs"]
    idx = sk["idx"]
    inputs_dict["alg_kwargs"]["alg_seed"] = sk["algorithm_seed"]
    inputs_dict["alg_kwargs"]["save_path"] = sk.get("save_path", "./logs")
    env_kwargs = inputs_dict["env_kwargs"]
    init_seeds(sk["setup_seed"])
    env, env_eval, env_expert = init_env(**env_kwargs), init_env(**env_kwargs), init_env(**env_kwargs)
    ak = dict(inputs_dict["actor_kwargs"])
    ak.setdefault("actor_weights", None)
    actor = init_actor(env, **ak)
    expert_kwargs = dict(ak)
    expert_kwargs["actor_weights"] = None
    if sk.get("expert_file") is not None:
        raise NotImplementedError("expert_file import reads a pickle; load expert weights with set_weights instead")
    expert = init_actor(env, **expert_kwargs)
    ck = dict(inputs_dict["critic_kwargs"])
    ck.setdefault("critic_weights", None)
    critics, q_targets, q_critics = init_critics(env, **ck)
    mk = dict(inputs_dict["model_kwargs"])
    for k in ("model_weights", "reward_weights"):
        mk.setdefault(k, None)
    models = init_world_models(env, **mk, model_setup_kwargs=inputs_dict["model_setup_kwargs"])
    init_seeds(sk["eval_seed"], env_eval)
    init_seeds(sk["sim_seed"], env)
    init_seeds(sk["expert_seed"], env_expert)
    alg = init_alg(idx, env, env_eval, env_expert, actor, critics, q_targets, q_critics, models,
                   inputs_dict["alg_kwargs"], inputs_dict["mf_update_kwargs"], expert, None)
    return alg.train(inputs_dict["alg_kwargs"]["total_timesteps"], inputs_dict)


def main(argv=None):
    start = datetime.now()
    args = create_train_parser().parse_args(argv)
    inputs_dict = gather_inputs(args)
    if args.alg_type in ("sac", "sac_imit"):
        inputs_dict["actor_kwargs"]["actor_squash"] = True     # SAC uses the squashed actor
    seeds = derive_seeds(args.seed, args.runs, args.runs_start)
    runs = list(range(args.runs))
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws > 1:
        import torch
        rank, local = int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        runs = runs[rank::ws]
    names = []
    for r in runs:
        d = {g: dict(v) for g, v in inputs_dict.items()}
        d["setup_kwargs"].update(idx=args.runs_start + r, setup_seed=int(seeds["setup"][r]),
                                 sim_seed=int(seeds["sim"][r]), eval_seed=int(seeds["eval"][r]),
                                 expert_seed=int(seeds["expert"][r]), algorithm_seed=int(seeds["algorithm"][r]))
        names.append(train(d))
    print(f"done: {names} in {(datetime.now() - start).total_seconds():.1f}s", flush=True)
    return names


if __name__ == "__main__":
    sys.exit(0 if main() else 1)
