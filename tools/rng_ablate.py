"""Is the sampler on the critical path?  Graph time per update with and without k_rng
(sacx_time_graph ablation: the skipped sampler leaves stale randoms, timing only)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "sac-expert_amd"))


def main():
    import bench
    from sac_eo.common.replicas import init_replica
    rep = init_replica()
    for cfg in sys.argv[1:] or ["hc"]:
        eng = bench.build_engine(bench.CONFIGS[cfg], rep.seeds(0), rep.device)
        eng.step(256)
        eng.sync()
        full = eng.time_graph(10)
        wo = eng.time_graph(10, "k_rng")
        prof = eng.profile(5)
        info = eng.plan_info()
        rng_us = [p * 1e3 for p, L in zip(prof, info) if L["kernel"] == "k_rng"]
        print(f"{cfg}: graph {full * 1e3:.1f} us/update, without k_rng {wo * 1e3:.1f} us/update, "
              f"eager k_rng {rng_us} us", flush=True)
        eng.close()


if __name__ == "__main__":
    main()
