"""Where the drop-in loop's time goes (diagnostic): act(1 obs) -> host, append(1), step(1),
each timed alone over n iterations, then the combined iteration (bench.drop_in_loop)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "sac-expert_amd"))


def main():
    import torch
    import bench
    from sac_eo.common.replicas import init_replica
    rep = init_replica()
    cfgd = bench.CONFIGS["hc"]
    eng = bench.build_engine(cfgd, bench.replica_seeds(rep, 1), rep.device)
    S, A = cfgd["S"], cfgd["A"]
    obs = torch.randn(1, S, device=eng.device)
    sp = torch.randn(1, S, device=eng.device)
    a_dev = torch.zeros(1, A, device=eng.device)
    z = torch.zeros(1)
    eng.prepare(1)
    n = 300

    def timed(name, fn):
        for j in range(10):
            fn(j)
        eng.sync()
        t0 = time.perf_counter()
        for j in range(n):
            fn(j)
        eng.sync()
        print(f"{name:40s} {(time.perf_counter() - t0) / n * 1e6:8.1f} us")

    timed("act -> host", lambda j: eng.act(obs, deterministic=False).cpu())
    timed("act (device only)", lambda j: eng.act(obs, deterministic=False))
    timed("append (host r, d)", lambda j: eng.append(obs, a_dev, z, sp, z))
    timed("append (device)", lambda j: eng.append(obs, a_dev, a_dev[:, 0], sp, a_dev[:, 0]))
    import numpy as np
    on, rn = np.zeros(S, np.float32), np.zeros(1, np.float32)
    timed("act (host obs) -> host, torch", lambda j: eng.act(on, deterministic=False).cpu().numpy())
    timed("act_host (C pinned staging)", lambda j: eng.act_host(on, deterministic=False))
    timed("append (all host, C staging)", lambda j: eng.append(on[None], np.zeros((1, A), np.float32), rn, on[None], rn))
    timed("step(1)", lambda j: eng.step(1, num_timesteps=j, ts_increment=1))
    timed("step(1) + sync", lambda j: (eng.step(1, num_timesteps=j, ts_increment=1), eng.sync()))
    print(bench.drop_in_loop(eng, cfgd))


if __name__ == "__main__":
    main()
