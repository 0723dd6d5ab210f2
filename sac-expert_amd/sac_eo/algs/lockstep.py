"""K learners of one packed handle trained in lock-step: the reference's ``--runs K``
(sac_eo/train.py:118-152 runs them as K processes) as K seeds of ONE libsacx handle.

Each learner's ``_train_loop`` (SACBase) yields the three requests of a timestep -- act, update,
add -- and does everything else itself on its own seed (SeedView: episode hooks, model fits,
diagnostics, logs, checkpoints).  This driver answers a round of K identical requests with ONE
launch chain for all seeds: ``sacx_actor_act_host_seeds`` (each seed's actor, normaliser and
stream), ``sacx_sac_step`` (the packed update graph, grid z = seed) and
``sacx_buffer_append_host_seeds``.  Every seed computes exactly what its one-seed run computes
(packed == single is bit-identical), so each run's log equals its serial run's.

Lock-step needs the K loops to ask for the same update schedule: SAC_exp updates once per env
step whatever the episode boundaries; SAC's G updates every real_step_mod steps of an episode
need episodes of equal length (no early termination).  A divergence raises."""
import os
import time

import numpy as np


def run_lockstep(algs, engine, total_timesteps, params_list):
    """Trains every learner of ``algs`` (one per seed of the packed ``engine``, seed order);
    returns their checkpoint names."""
    if len(algs) != engine.seeds:
        raise ValueError("one learner per seed of the packed handle")
    loops = [a._train_loop(total_timesteps, p) for a, p in zip(algs, params_list)]
    reqs = [next(lp) for lp in loops]
    names = [None] * len(loops)
    K = len(loops)
    obs_buf = add_buf = None        # one round's rows, filled in place (no np.stack per round)
    prof = {} if os.environ.get("SACX_LOCKSTEP_PROFILE") else None   # seconds per phase (diagnostic)
    while True:
        kind = reqs[0][0]
        t0 = time.perf_counter() if prof is not None else 0.0
        if any(r[0] != kind for r in reqs):
            raise RuntimeError("packed runs diverged: the learners ask for different steps "
                               "(use --serial_runs)")
        if kind == "act":
            det = reqs[0][2]
            if any(r[2] != det for r in reqs):
                raise RuntimeError("packed runs diverged: deterministic and stochastic actions in one round")
            shp = np.shape(reqs[0][1])
            if obs_buf is None or obs_buf.shape[1:] != shp:
                obs_buf = np.empty((K,) + shp, np.float32)
            for i, r in enumerate(reqs):
                obs_buf[i] = r[1]
            outs = engine.act_host_seeds(obs_buf, deterministic=det)
            results = list(outs)
        elif kind == "update":
            if any(tuple(r[1:]) != tuple(reqs[0][1:]) for r in reqs):
                raise RuntimeError("packed runs diverged: different update schedules (episodes of different "
                                   "length under SAC's real_step_mod; use --serial_runs)")
            engine.step(reqs[0][1], num_timesteps=reqs[0][2], ts_increment=reqs[0][3])
            results = [None] * len(reqs)
        elif kind == "add":
            shps = [np.shape(reqs[0][1][j]) for j in range(5)]
            if add_buf is None or [b.shape[1:] for b in add_buf] != shps:
                add_buf = [np.empty((K,) + sh, np.float32) for sh in shps]
            for i, r in enumerate(reqs):
                for j in range(5):
                    add_buf[j][i] = r[1][j]
            n = engine.append_host_seeds(*add_buf)
            results = [n] * len(reqs)
        else:
            raise ValueError(kind)
        if prof is not None:
            t1 = time.perf_counter()
            prof[kind] = prof.get(kind, 0.0) + (t1 - t0)
        finished = 0
        for i, (lp, res) in enumerate(zip(loops, results)):
            try:
                reqs[i] = lp.send(res)
            except StopIteration as stop:
                names[i] = stop.value
                finished += 1
        if prof is not None:
            prof["learners after " + kind] = prof.get("learners after " + kind, 0.0) + (time.perf_counter() - t1)
        if finished == len(loops):
            if prof is not None:
                print("lockstep phases (s): " + ", ".join(f"{k} {v:.3f}" for k, v in sorted(prof.items())), flush=True)
            return names
        if finished:
            raise RuntimeError("packed runs diverged: some learners finished before the others")
