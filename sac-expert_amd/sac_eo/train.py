"""``python -m sac_eo.train`` (reference ``sac_eo/train.py``): same flags, seeds and
construction sequence, one learner per process, the same log files.

Runs are spread over processes: under ``torch.distributed.run`` rank r trains runs
``r, r + world, ...`` on its local GPU.  The runs of one process train as K packed seeds of
ONE device handle in lock-step (sac_eo.algs.lockstep: one launch chain per timestep for all
of them, each run's log identical to its serial run's), or -- with ``--serial_runs``, or where
lock-step cannot hold (SAC with early-terminating episodes, ``--env_batch_type traj``,
``--actor_layer_norm``) -- one after another.  No data moves between learners (SURVEY §8e:
replicas).  As in the reference (``:159-191``), the runs' checkpoint logs are gathered into one
pickled list ``<env_type>_<env>_<alg_type>_<mf_algo>[_<save_file>]_<date>`` and removed."""
import copy
import os
import pickle
import sys
from datetime import datetime

import numpy as np

from .actors import init_actor
from .algs import init_alg
from .common.seeding import derive_seeds, init_seeds
from .common.logger import load_log
from .common.train_parser import create_train_parser, gather_inputs
from .common.train_utils import import_inputs, load_expert
from .critics import init_critics
from .envs import init_env
from .models import init_world_models


def build_alg(inputs_dict, pack=None):
    """The construction sequence of one run (reference train.py:33-103); pack = (shared packed
    Engine or None, seed, K) makes the learner one seed of a packed handle."""
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
    if sk.get("expert_file") is not None:        # train.py:65-86
        expert_kwargs, init_expert_rms_stats = load_expert(sk["expert_path"], sk["expert_file"])
    else:
        expert_kwargs = dict(ak)
        expert_kwargs["actor_weights"] = None
        init_expert_rms_stats = None
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
    if pack is not None:
        inputs_dict["alg_kwargs"]["_pack"] = pack
    return init_alg(idx, env, env_eval, env_expert, actor, critics, q_targets, q_critics, models,
                    inputs_dict["alg_kwargs"], inputs_dict["mf_update_kwargs"], expert, init_expert_rms_stats)


def train(inputs_dict):
    """Training on one seed (reference train.py:33-107)."""
    alg = build_alg(inputs_dict)
    return alg.train(inputs_dict["alg_kwargs"]["total_timesteps"], inputs_dict)


def lockstep_ok(args, env_kwargs, k: int) -> bool:
    """Whether k runs of a process can train as packed seeds in lock-step (sac_eo.algs.lockstep):
    one row per run and request must fit the library's pinned staging (SACX_STAGE_FLOATS)."""
    if args.serial_runs or args.alg_type not in ("sac", "sac_imit") or args.env_batch_type != "steps":
        return False
    if args.actor_layer_norm:
        return False
    env = init_env(**env_kwargs)
    S, A = int(np.prod(env.observation_space.shape)), int(np.prod(env.action_space.shape))
    from ._native import STAGE_FLOATS
    if k * (2 * S + A + 2) > STAGE_FLOATS or k * (S + A) > STAGE_FLOATS:
        return False
    if args.alg_type == "sac":            # G updates every real_step_mod steps of an EPISODE
        return getattr(env, "terminate", True) is False
    return True


def train_packed(inputs_list):
    """The runs of ``inputs_list`` as seeds of one packed handle, in lock-step."""
    from .algs.lockstep import run_lockstep
    algs, shared = [], None
    for i, d in enumerate(inputs_list):
        alg = build_alg(d, pack=(shared, i, len(inputs_list)))
        shared = shared if shared is not None else alg.engine._eng
        algs.append(alg)
    return run_lockstep(algs, shared, inputs_list[0]["alg_kwargs"]["total_timesteps"], inputs_list)


def _train_runs(runs, run_inputs, args, local_rank=None):
    """One process's share of the runs: lock-step packed seeds of one handle where that holds,
    else one after another.  Returns {run: checkpoint name}."""
    if local_rank is not None:
        import torch
        torch.cuda.set_device(local_rank)
    if len(runs) > 1 and lockstep_ok(args, run_inputs[0]["env_kwargs"], len(runs)):
        return dict(zip(runs, train_packed(run_inputs)))
    return {r: train(d) for r, d in zip(runs, run_inputs)}


def _pool_worker(job):
    runs, run_inputs, args, local_rank = job
    return _train_runs(runs, run_inputs, args, local_rank)


def pool_size(args, n_runs: int) -> int:
    """Processes per GPU for the runs of one rank: the reference's Pool(--cores) (train.py:148-152),
    capped by the usable host cores and by MAX_PROCS_PER_GPU (each process holds its own device
    context and arena); each process trains its runs as packed seeds.  Without --cores: ONE process
    per GPU packing all of its runs -- not the reference's one process per run: processes sharing a
    GPU time-slice it (8 HC runs of sac: packed 3.02x serial, 2 / 4 / 8 processes 1.46x / 0.72x /
    0.73x; profiles/r04_packed_runs_sac_v1.log)."""
    want = args.cores if args.cores is not None else 1
    usable = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    return max(1, min(want, n_runs, usable, MAX_PROCS_PER_GPU))


MAX_PROCS_PER_GPU = int(os.environ.get("SACX_MAX_PROCS_PER_GPU", "4"))


def main(argv=None):
    start = datetime.now()
    args = create_train_parser().parse_args(argv)
    inputs_dict = gather_inputs(args)
    if args.alg_type in ("sac", "sac_imit"):
        inputs_dict["actor_kwargs"]["actor_squash"] = True     # SAC uses the squashed actor
    seeds = derive_seeds(args.seed, args.runs, args.runs_start)
    runs = list(range(args.runs))
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    local = None
    if ws > 1:
        rank, local = int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0"))
        runs = runs[rank::ws]
    names, run_inputs = {}, []
    for r in runs:
        d = copy.deepcopy(inputs_dict)
        # train.py:132-142: a seed given on the command line is kept, the others derived per run
        # (--alg_seed, which the reference never stores and then fails on, is used as given)
        sk = d["setup_kwargs"]
        sk["idx"] = args.runs_start + r
        for kind, key in (("setup", "setup_seed"), ("sim", "sim_seed"), ("eval", "eval_seed"),
                          ("expert", "expert_seed")):
            if sk.get(key) is None:
                sk[key] = int(seeds[kind][r])
        sk["algorithm_seed"] = int(seeds["algorithm"][r]) if args.alg_seed is None else int(args.alg_seed)
        run_inputs.append(import_inputs(d))          # train_utils.py:20-92 (no-op without --import_file)
    P = pool_size(args, len(runs))
    if P > 1:
        # the reference's process pool (train.py:151-152): P spawned processes share this GPU, each
        # with runs r, r + P, ... as lock-step packed seeds; this process never touches the GPU
        import multiprocessing as mp
        jobs = [(runs[i::P], run_inputs[i::P], args, local) for i in range(P)]
        with mp.get_context("spawn").Pool(P) as pool:
            for part in pool.map(_pool_worker, jobs):
                names.update(part)
    else:
        names = _train_runs(runs, run_inputs, args, local)
    if ws > 1:                                       # every rank's runs are on disk before gathering
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        from datetime import timedelta
        # ranks may finish their runs far apart: no collective timeout in the gathering group
        dist.init_process_group("gloo", rank=rank, world_size=ws, timeout=timedelta(days=7))
        dist.barrier()
        allnames = [None] * ws
        dist.all_gather_object(allnames, names)
        dist.destroy_process_group()
        if rank != 0:
            return None
        names = {k: v for part in allnames for k, v in part.items()}
    # gather the runs' logs into one file, in run order (train.py:159-191)
    outputs = [load_log(os.path.join(args.save_path, names[r])) for r in sorted(names)]
    save_env = args.env_name.split("-")[0].lower()
    if args.task_name is not None:
        save_env = f"{save_env}_{args.task_name.lower()}"
    date = datetime.today().strftime("%m%d%y_%H%M%S")
    parts = [args.env_type.lower(), save_env, args.alg_type, args.mf_algo] + \
        ([args.save_file] if args.save_file is not None else []) + [date]
    save_filefull = os.path.join(args.save_path, "_".join(parts))
    with open(save_filefull, "wb") as fh:
        pickle.dump(outputs, fh, protocol=4)
    for r in sorted(names):
        os.remove(os.path.join(args.save_path, names[r]))
    print(f"done: {save_filefull} in {(datetime.now() - start).total_seconds():.1f}s", flush=True)
    return save_filefull


if __name__ == "__main__":
    main()
    sys.exit(0)
