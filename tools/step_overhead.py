"""Fixed cost of one sacx_sac_step(n) call at the bench's hc config: host time of the launch call
(graph replay enqueue) and of launch + synchronize for n updates, median over repeats, and the
least-squares line t(n) = a + b n over the sizes.  The driver times step(20): a is what a 20-update
region pays on top of 20 steady-state updates (sampler start-up, alpha tail, launch + wake-up).
Usage: step_overhead.py [sizes comma-sep] [repeats]."""
import os
import sys
import time

sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "sac-expert_amd")]

import numpy as np   # noqa: E402


def bench_order(order, steps=20, warmup=5):
    """The bench's own sequence in a fresh process: order "warmup-prepare" (warmup, then the
    untimed graph capture, then the timed call) or "prepare-warmup" (capture first, so the timed
    call follows the warmup's GPU work directly)."""
    import bench
    from sac_eo.common.replicas import init_replica
    rep = init_replica()
    eng = bench.build_engine(bench.CONFIGS["hc"], rep.seeds(0), device=rep.device)
    if os.environ.get("EXTERNAL"):             # experiment: single-stream graphs (no sampler branch)
        step0 = eng.step
        eng.step = lambda n, **kw: step0(n, external=True, **kw)
        prep0 = eng.prepare
        eng.prepare = lambda n: prep0(n, external=True)
    if order == "prepare-warmup":
        eng.prepare(steps)
        eng.sync()
    eng.step(warmup, num_timesteps=0, ts_increment=1)
    if order == "warmup-prepare":
        eng.prepare(steps)
    if os.environ.get("PRE_STEPS"):           # experiment: more updates on warm graphs just before
        eng.step(int(os.environ["PRE_STEPS"]), num_timesteps=0, ts_increment=1)
    eng.sync()
    if os.environ.get("SPIN_MS"):             # experiment: a non-learner GPU load before the region
        import torch
        x = torch.randn(4096, 4096, device=rep.device)
        t_end = time.perf_counter() + float(os.environ["SPIN_MS"]) * 1e-3
        while time.perf_counter() < t_end:
            x = x @ x
            x = x / x.norm()
            torch.cuda.synchronize()
    rep.barrier()
    t0 = time.perf_counter()
    eng.step(steps, num_timesteps=warmup, ts_increment=1)
    tl = time.perf_counter() - t0
    eng.sync()
    el = time.perf_counter() - t0
    t0 = time.perf_counter()
    eng.step(steps, num_timesteps=warmup, ts_increment=1)
    tl2 = time.perf_counter() - t0
    eng.sync()
    el2 = time.perf_counter() - t0
    print(f"{order} spin {os.environ.get('SPIN_MS', '0')} ms: {el * 1e6:8.1f} us = {steps / el:9.1f} updates/s "
          f"(launch call {tl * 1e6:7.1f} us); a second call {el2 * 1e6:8.1f} us (launch {tl2 * 1e6:7.1f} us)",
          flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] in ("warmup-prepare", "prepare-warmup"):
        bench_order(sys.argv[1])
        return
    sizes = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [1, 2, 5, 10, 20, 40, 80, 160]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    import bench
    from sac_eo.common.replicas import init_replica
    rep = init_replica()
    eng = bench.build_engine(bench.CONFIGS["hc"], rep.seeds(0), device=rep.device)
    eng.step(5, num_timesteps=0, ts_increment=1)
    rows = []
    for n in sizes:
        eng.prepare(n)
        eng.sync()
        tl, tt = [], []
        for _ in range(reps):
            t0 = time.perf_counter()
            eng.step(n, num_timesteps=5, ts_increment=1)
            t1 = time.perf_counter()
            eng.sync()
            t2 = time.perf_counter()
            tl.append(t1 - t0)
            tt.append(t2 - t0)
        ml, mt = np.median(tl) * 1e6, np.median(tt) * 1e6
        rows.append((n, ml, mt, np.min(tt) * 1e6))
        print(f"n={n:4d} launch {ml:8.1f} us  total {mt:9.1f} us (min {np.min(tt) * 1e6:9.1f})  "
              f"{mt / n:7.2f} us/update  {n / mt * 1e6:9.1f} updates/s", flush=True)
    n = np.array([r[0] for r in rows], float)
    t = np.array([r[2] for r in rows])
    b, a = np.polyfit(n, t, 1)
    print(f"fit: total = {a:.1f} us + {b:.2f} us x n  (n=20 predicted {a + 20 * b:.1f} us)")
    # the bench's timed region is ONE call after an idle gap (prepare, sync, barrier): what a
    # first replay of a fresh graph, and a replay after the GPU idled, cost on top of a warm loop
    def once(m, pause):
        eng.sync()
        if pause:
            time.sleep(pause)
        t0 = time.perf_counter()
        eng.step(m, num_timesteps=5, ts_increment=1)
        eng.sync()
        return (time.perf_counter() - t0) * 1e6
    for m in (21, 23, 27):
        eng.prepare(m)
        eng.sync()
        first = once(m, 0.0)
        warm = [once(m, 0.0) for _ in range(5)]
        print(f"n={m}: first replay of a fresh graph {first:8.1f} us, then {np.median(warm):8.1f} us")
    for pause in (0.0, 0.001, 0.01, 0.1, 0.5):
        v = [once(20, pause) for _ in range(7)]
        print(f"n=20 after {pause * 1e3:6.1f} ms idle: median {np.median(v):8.1f} us  min {np.min(v):8.1f}", flush=True)


if __name__ == "__main__":
    main()
