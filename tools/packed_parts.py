"""Where a lock-step --runs iteration's time goes (diagnostic): K packed seeds (single_seed_plan,
as sac_eo.train builds them), act_host_seeds / step(1) / append_host_seeds each timed alone over
n iterations, then the combined iteration.  Usage: packed_parts.py [K] [single_seed_plan 0/1]."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sac-expert_amd")]


def main():
    import numpy as np
    import torch
    from sac_eo.engine import Engine, EngineConfig
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    ssp = bool(int(sys.argv[2])) if len(sys.argv) > 2 else True
    S, A = 17, 6
    eng = Engine(EngineConfig(s_dim=S, a_dim=A, batch=256, buffer_capacity=100_000, seeds=K,
                              single_seed_plan=ssp, graph_steps=128))
    rs = np.random.RandomState(0)
    rows = [rs.normal(size=(K, 2000, S)).astype(np.float32), rs.normal(size=(K, 2000, A)).astype(np.float32),
            rs.normal(size=(K, 2000)).astype(np.float32), rs.normal(size=(K, 2000, S)).astype(np.float32),
            np.zeros((K, 2000), np.float32)]
    for c in range(0, 2000, 150):                         # within the pinned staging buffer
        eng.append_host_seeds(*[x[:, c:c + 150] for x in rows])
    obs = rs.normal(size=(K, S)).astype(np.float32)
    one = [rows[0][:, :1], rows[1][:, :1], rows[2][:, :1], rows[3][:, :1], rows[4][:, :1]]
    eng.prepare(1)
    n = 200

    def timed(name, fn):
        for j in range(5):
            fn(j)
        eng.sync()
        t0 = time.perf_counter()
        for j in range(n):
            fn(j)
        eng.sync()
        print(f"{name:36s} {(time.perf_counter() - t0) / n * 1e6:8.1f} us", flush=True)

    timed("act_host_seeds (deterministic)", lambda j: eng.act_host_seeds(obs, deterministic=True))
    timed("act_host_seeds (stochastic)", lambda j: eng.act_host_seeds(obs, deterministic=False))
    timed("append_host_seeds", lambda j: eng.append_host_seeds(*one))
    timed("step(1)", lambda j: eng.step(1, num_timesteps=j, ts_increment=1))
    timed("iteration act -> step(1) -> append", lambda j: (eng.act_host_seeds(obs, deterministic=True),
                                                          eng.step(1, num_timesteps=j, ts_increment=1),
                                                          eng.append_host_seeds(*one)))
    eng.close()


if __name__ == "__main__":
    main()
