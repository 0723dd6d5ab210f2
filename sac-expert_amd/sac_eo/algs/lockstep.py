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
import numpy as np


def run_lockstep(algs, engine, total_timesteps, params_list):
    """Trains every learner of ``algs`` (one per seed of the packed ``engine``, seed order);
    returns their checkpoint names."""
    if len(algs) != engine.seeds:
        raise ValueError("one learner per seed of the packed handle")
    loops = [a._train_loop(total_timesteps, p) for a, p in zip(algs, params_list)]
    reqs = [next(lp) for lp in loops]
    names = [None] * len(loops)
    while True:
        kind = reqs[0][0]
        if any(r[0] != kind for r in reqs):
            raise RuntimeError("packed runs diverged: the learners ask for different steps "
                               "(use --serial_runs)")
        if kind == "act":
            det = reqs[0][2]
            if any(r[2] != det for r in reqs):
                raise RuntimeError("packed runs diverged: deterministic and stochastic actions in one round")
            outs = engine.act_host_seeds(np.stack([np.asarray(r[1], np.float32) for r in reqs]), deterministic=det)
            results = list(outs)
        elif kind == "update":
            if any(tuple(r[1:]) != tuple(reqs[0][1:]) for r in reqs):
                raise RuntimeError("packed runs diverged: different update schedules (episodes of different "
                                   "length under SAC's real_step_mod; use --serial_runs)")
            engine.step(reqs[0][1], num_timesteps=reqs[0][2], ts_increment=reqs[0][3])
            results = [None] * len(reqs)
        elif kind == "add":
            f = [np.stack([r[1][i] for r in reqs]) for i in range(5)]
            n = engine.append_host_seeds(*f)
            results = [n] * len(reqs)
        else:
            raise ValueError(kind)
        finished = 0
        for i, (lp, res) in enumerate(zip(loops, results)):
            try:
                reqs[i] = lp.send(res)
            except StopIteration as stop:
                names[i] = stop.value
                finished += 1
        if finished == len(loops):
            return names
        if finished:
            raise RuntimeError("packed runs diverged: some learners finished before the others")
