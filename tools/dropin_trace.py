"""Device timeline of the drop-in loop (diagnostic): run bench.drop_in_loop at the hc config (under
rocprofv3 --kernel-trace --memory-copy-trace), or, given the trace directory, cut the timeline into
iterations at the behaviour-action kernel and report where each iteration's time goes: kernel busy
time, the idle gaps and the launches on either side of each gap.

  rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d DIR -o d -- python tools/dropin_trace.py run
  python tools/dropin_trace.py DIR"""
import csv
import glob
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "sac-expert_amd"))


def run():
    import bench
    from sac_eo.common.replicas import init_replica
    rep = init_replica()
    cfgd = bench.CONFIGS["hc"]
    eng = bench.build_engine(cfgd, bench.replica_seeds(rep, 1), rep.device)
    eng.step(50, num_timesteps=0, ts_increment=1)
    eng.sync()
    r = bench.drop_in_loop(eng, cfgd, n=int(os.environ.get("DROPIN_N", "200")))
    print(r)


def host():
    """Host time of each call of the drop-in iteration (no profiler): act_host (returns once the
    action is on the host), step(1) and append (enqueue only), means over the iterations."""
    import time
    import numpy as np
    import bench
    from sac_eo.common.replicas import init_replica
    rep = init_replica()
    cfgd = bench.CONFIGS["hc"]
    eng = bench.build_engine(cfgd, bench.replica_seeds(rep, 1), rep.device)
    S, A = cfgd["S"], cfgd["A"]
    rs = np.random.RandomState(0)
    obs = [rs.normal(size=S).astype(np.float32) for _ in range(16)]
    r1, d1 = np.zeros(1, np.float32), np.zeros(1, np.float32)
    eng.prepare(1)
    n = 400
    acc = np.zeros(4)
    for j in range(n + 20):
        o, o2 = obs[j % 16], obs[(j + 1) % 16]
        t0 = time.perf_counter()
        a = eng.act_host(o, deterministic=True)
        t1 = time.perf_counter()
        eng.step(1, num_timesteps=j, ts_increment=1)
        t2 = time.perf_counter()
        eng.append(o[None], a[None], r1, o2[None], d1)
        t3 = time.perf_counter()
        if j >= 20:
            acc += np.array([t1 - t0, t2 - t1, t3 - t2, t3 - t0])
    eng.sync()
    acc *= 1e6 / n
    print(f"host us per call: act_host {acc[0]:.2f}  step(1) {acc[1]:.2f}  append {acc[2]:.2f}  iteration {acc[3]:.2f}")


def short(name):
    n = name.split("(")[0].replace("void ", "").replace("sacx::", "")
    return n[:44]


def analyse(d):
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    ev = []
    for r in csv.DictReader(open(kt)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    for mc in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
        for r in csv.DictReader(open(mc)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy " + r.get("Direction", "?")))
    ev.sort()
    marks = [i for i, e in enumerate(ev) if "act" in e[2] and "k_act" in e[2]]
    if len(marks) < 20:
        print("too few act kernels:", len(marks))
        return
    its = list(zip(marks[-101:-1], marks[-100:]))
    tot = busy = 0.0
    gaps = {}
    per_kernel = {}
    for a, b in its:
        t0, t1 = ev[a][0], ev[b][0]
        tot += (t1 - t0) / 1e3
        cur = t0
        for i in range(a, b):
            s, e, n = ev[i]
            if s > cur:
                key = (ev[i - 1][2] if i > a else "<start>") + " -> " + n
                g = gaps.setdefault(key, [0.0, 0])
                g[0] += (s - cur) / 1e3
                g[1] += 1
            busy += max(0, e - max(s, cur)) / 1e3
            cur = max(cur, e)
            k = per_kernel.setdefault(n, [0.0, 0])
            k[0] += (e - s) / 1e3
            k[1] += 1
    n = len(its)
    print(f"{n} iterations: {tot / n:.2f} us each, GPU busy {busy / n:.2f} us, idle {(tot - busy) / n:.2f} us")
    print("\nlaunches per iteration (mean duration, us):")
    for k, (t, c) in sorted(per_kernel.items(), key=lambda kv: -kv[1][0]):
        print(f"  {k:46s} {c / n:5.2f} x {t / c:7.2f}")
    print("\nidle gaps per iteration (us, before -> after):")
    for k, (t, c) in sorted(gaps.items(), key=lambda kv: -kv[1][0])[:16]:
        print(f"  {t / n:7.2f}  ({c / n:4.2f} x {t / c:6.2f})  {k}")
    print("\none iteration's timeline (us from the action kernel's start):")
    a, b = its[-1]
    for i in range(a, b + 1):
        s, e, nm = ev[i]
        print(f"  {(s - ev[a][0]) / 1e3:8.2f} {(e - ev[a][0]) / 1e3:8.2f}  {nm}")


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "run":
        run()
    elif len(sys.argv) > 1 and sys.argv[1] == "host":
        host()
    else:
        analyse(sys.argv[1])
