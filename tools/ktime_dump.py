"""Per-launch workgroup timing of one update-graph replay (diagnostic).

Runs bench.py's engine, replays the timed graph once with SACX_KTIME_DUMP set and prints,
per k_gemm launch: workgroups, launch span, mean / max workgroup duration, the offset of
the last workgroup start (dispatch skew) and the gap after the previous k_gemm launch."""
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "sac-expert_amd"))


def main():
    import bench
    from sac_eo.common.replicas import init_replica
    cfg = sys.argv[1] if len(sys.argv) > 1 else "hc"
    rep = init_replica()
    k = int(os.environ.get("KT_SEEDS", "1"))           # packed seeds per handle
    eng = bench.build_engine(bench.CONFIGS[cfg], bench.replica_seeds(rep, k), rep.device)
    eng.step(300)
    eng.sync()
    path = os.path.join(tempfile.mkdtemp(), "kt.csv")
    os.environ["SACX_KTIME_DUMP"] = path
    cpath = os.path.join(os.path.dirname(path), "kc.csv")
    os.environ["SACX_KTIME_CLASSES"] = cpath
    eng.time_kernels("k_gemm", 2)
    rows = [l.strip().split(",") for l in open(path)]
    G = eng.cfg.graph_steps
    per = len(rows) // G
    mid = rows[(G // 2) * per:(G // 2 + 1) * per]      # one update from the middle of the graph
    print(f"{'launch':34s} {'WGs':>5s} {'span':>6s} {'wg_avg':>6s} {'wg_max':>6s} {'skew':>6s} {'gap':>6s}")
    for r in mid:
        print(f"{r[0]:34s} {r[1]:>5s} {r[2]:>6s} {r[3]:>6s} {r[4]:>6s} {r[5]:>6s} {r[6]:>6s}")
    import numpy as np
    # per launch name, averaged over every update of the graph
    agg = {}
    for r in rows:
        agg.setdefault(r[0], []).append([float(x) for x in r[2:]])
    print(f"\n{'launch (mean over updates)':34s} {'n':>5s} {'span':>6s} {'wg_avg':>6s} {'wg_max':>6s} {'skew':>6s} "
          f"{'gap':>6s} {'row_avg':>7s} {'row_max':>7s} {'gap_med':>7s} {'gap_p90':>7s}")
    for name, v in agg.items():
        va = np.array(v)
        v = va.mean(0)
        print(f"{name:34s} {len(agg[name]):5d} {v[0]:6.2f} {v[1]:6.2f} {v[2]:6.2f} {v[3]:6.2f} {v[4]:6.2f} "
              f"{v[5]:7.2f} {v[6]:7.2f} {np.median(va[:, 4]):7.2f} {np.percentile(va[:, 4], 90):7.2f}")
    # k_fwd2 launches: workgroups per problem pair (n:mean:max us), averaged over the graph's updates
    cls = {}
    if os.path.exists(cpath):
        for l in open(cpath):
            f = l.strip().split(",")
            cls.setdefault(f[0], []).append([[float(x) for x in c.split(":")[1:]] for c in f[1:]])
    if cls:
        print(f"\n{'k_fwd2 launch: tiles per problem pair':34s} n / mean / max us")
        for name, v in cls.items():
            v = np.array(v).mean(0)
            print(f"{name:34s} " + "  ".join(f"p{i}: {int(c[0])} / {c[1]:.2f} / {c[2]:.2f}" for i, c in enumerate(v)))
    a = np.array([[float(x) for x in r[2:]] for r in rows])
    print(f"mean over {len(rows)} launches: span {a[:, 0].mean():.2f} wg_avg {a[:, 1].mean():.2f} "
          f"wg_max {a[:, 2].mean():.2f} skew {a[:, 3].mean():.2f} gap {a[:, 4].mean():.2f} us")
    eng.close()


if __name__ == "__main__":
    main()
