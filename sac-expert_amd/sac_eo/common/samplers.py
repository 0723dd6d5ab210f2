"""trajectory_sampler (reference ``sac_eo/common/samplers.py:3-70``)."""
import numpy as np


def trajectory_sampler(env, actor, horizon, s_init=None, eval=False, deterministic=False, corruptor=None):
    s_traj, a_traj, r_traj, sp_traj, d_traj = [], [], [], [], []
    J_tot = 0.0
    s = env.reset(s_init) if s_init is not None else env.reset()
    for t in range(horizon):
        s_old = s
        a = actor.sample(s_old, deterministic=deterministic).numpy()
        s_true, r, d, _ = env.step(actor.clip(a))
        s_store, s = corruptor.store_and_next(s_true) if corruptor is not None else (s_true, s_true)
        if eval:
            J_tot += r
        if t == horizon - 1:
            d = False
        s_traj.append(s_old)
        a_traj.append(a)
        r_traj.append(r)
        sp_traj.append(s_store)
        d_traj.append(d)
        if d:
            break
    out = (np.array(s_traj, np.float32), np.array(a_traj, np.float32), np.array(r_traj, np.float32),
           np.array(sp_traj, np.float32), np.array(d_traj))
    return out + (J_tot,) if eval else out
