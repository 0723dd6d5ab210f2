"""SAC gradient-steps/sec on MI355X (BASELINE.json metric, configs[1]).

Workload (default ``--config hc``): HalfCheetah-v3-shaped synthetic replay
buffer (obs 17, act 6, 1e6 rows resident in HBM), plain SAC twin-Q + actor +
alpha update (alg ``sac``, no world model), batch 256, 256x2 relu MLPs, fp32.
A step = one ``_update`` (SAC.py:236-250): sampler + gather, target, both
critic Adams, actor Adam, alpha Adam, Polyak.

Multi-GPU: one process per GPU (torch.distributed.run), each an independent
learner with its own seed -- the reference's ``--runs N`` spawn-pool
parallelism (train.py:118-152).  No data-path collective; ``value`` is the
sum of steps over ranks divided by the max-over-ranks wall time (weak scaling).

Packed seeds: ``--seeds-per-gpu K`` packs K independent learners into each
GPU's handle for the timed region (cfg.seeds = K: every launch of the update
graph runs all K, grid z = seed) and ``value`` counts every seed's updates.
The default keeps one learner per GPU and adds a ``packed_seeds`` leg (8 seeds
per GPU for hc) measured after the timed region.

Extra JSON fields: ``roofline`` for the dominant kernel (HIP-event timed in
this process) and ``cpu_baseline`` (the CPU oracle port on the host cores,
rank 0 at N=1, bounded sample).
"""
from __future__ import annotations

import argparse
import glob
import re
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "sac-expert_amd"))

CONFIGS = {
    # BASELINE.json configs[1]
    "hc": dict(workload="HalfCheetah-v3-shaped synthetic buffer, SAC twin-Q + actor + alpha update (no model), fp32",
               S=17, A=6, B=256, hidden=(256, 256), buffer=1_000_000, use_expert=False),
    # configs[0]-shaped: the reference's default algorithm (SAC-EO: expert term through two
    # 512x2 world models) at HalfCheetah shapes
    "hc_eo": dict(workload="HalfCheetah-v3-shaped synthetic buffer, SAC-EO update incl. world-model expert term, fp32",
                  S=17, A=6, B=256, hidden=(256, 256), buffer=1_000_000, use_expert=True),
    # configs[2]-shaped (SAC-EO expert term; model fitting is a separate call)
    "humanoid_eo": dict(workload="Humanoid-v3-shaped synthetic buffer, SAC-EO update incl. world-model expert term, fp32",
                        S=376, A=17, B=1024, hidden=(256, 256), buffer=1_000_000, use_expert=True),
    # configs[4] per replica: bf16 MFMA operands with fp32 accumulate, 4e6-row buffer in HBM
    "humanoid_bf16": dict(workload="Humanoid-v3-shaped synthetic 4e6-row buffer, SAC update, bf16 MFMA operands / "
                                   "fp32 accumulate and master weights",
                          S=376, A=17, B=1024, hidden=(256, 256), buffer=4_000_000, use_expert=False, bf16=True),
    # the same shapes in fp32 (the comparison point for humanoid_bf16)
    "humanoid_sac": dict(workload="Humanoid-v3-shaped synthetic 4e6-row buffer, SAC update, fp32",
                         S=376, A=17, B=1024, hidden=(256, 256), buffer=4_000_000, use_expert=False),
}

FP32_PEAK_TFLOPS = 157.3     # MI355X_MICROARCH.md: FP32 matrix (= vector) peak, dense
BF16_PEAK_TFLOPS = 2500.0    # dense BF16 MFMA (no sparsity)
HBM_PEAK_GBS = 8000.0


def build_engine(cfgd, seeds, device, dp=None, batch=None, weight_seed=None):
    """seeds: this replica's reference-style seeds (sac_eo.common.seeding.derive_seeds), one
    dict of scalars per learner; a list of K dicts builds a packed handle of K seeds (one launch
    chain for all, grid z = seed).  dp: (rccl id, ranks, rank) for the data-parallel mode, with
    the local `batch` and one `weight_seed` shared by all ranks (identical initial weights)."""
    import torch
    from sac_eo.engine import Engine, EngineConfig
    from sac_eo.nets import create_nn_weights
    seed_list = list(seeds) if isinstance(seeds, (list, tuple)) else [seeds]
    S, A = cfgd["S"], cfgd["A"]
    B = batch or cfgd["B"]
    ecfg = EngineConfig(s_dim=S, a_dim=A, hidden=cfgd["hidden"], activation="relu", batch=B,
                        buffer_capacity=cfgd["buffer"], use_expert=cfgd["use_expert"], expert_batch=20,
                        expert_capacity=20, graph_steps=int(os.environ.get("SACX_GRAPH_STEPS", "256")),
                        gemm_bf16=bool(cfgd.get("bf16", False)), seeds=len(seed_list))
    eng = Engine(ecfg, device=device, dp=dp)
    for k, sd in enumerate(seed_list):
        eng.select_seed(k)
        rng = np.random.default_rng(weight_seed if weight_seed is not None else sd["setup"])
        eng.set_net("actor", create_nn_weights(rng, S, A, cfgd["hidden"], 0.01))
        for j in range(2):
            w = create_nn_weights(rng, S + A, 1, cfgd["hidden"], 1.0)
            eng.set_net(f"q{j}", w)
            eng.set_net(f"t{j}", w)
        if cfgd["use_expert"]:
            for j in range(2):
                eng.set_net(f"m{j}", create_nn_weights(rng, S + A, S + 1, (512, 512), 0.01))
        # synthetic HalfCheetah-shaped rows generated on the device
        g = torch.Generator(device=device)
        g.manual_seed(int(sd["sim"]))                    # synthetic replay rows
        N = cfgd["buffer"]
        sig = torch.rand(S, device=device, generator=g) * 4.9 + 0.1
        s = torch.randn(N, S, device=device, generator=g) * sig
        sp = torch.randn(N, S, device=device, generator=g) * sig
        a = torch.rand(N, A, device=device, generator=g) * 2 - 1
        r = torch.randn(N, device=device, generator=g)
        d = torch.zeros(N, device=device)
        eng.append(s, a, r, sp, d)
        eng.sync()
        del s, sp, a, r, d
        if cfgd["use_expert"]:
            ers = np.random.RandomState(sd["eval"])
            eng.set_expert(ers.normal(size=(20, S)), ers.normal(size=(20, S)), 1e-3)
            gen = np.random.default_rng(sd["algorithm"])  # SAC_exp's self.rng (alg_seed)
            perms = np.stack([gen.permutation(20) for _ in range(4096)])
            eng.push_perms(perms)
        eng.rng_seed(sd["expert"])                     # global stream: last np.random.seed (train.py:95-97)
    eng.select_seed(0)
    eng.sync()
    return eng


def pmc_traffic(kernel, config):
    """HBM bytes per launch of `kernel` from the committed PMC summary of this config
    (tools/pmc_summary.py over tools/gpu_pmc.sh output: f x FETCH_SIZE + WRITE_SIZE, with the
    fetch factor f calibrated per access shape -- 2 for coalesced streaming reads, the gfx950
    correction of MI355X_MICROARCH.md section HBM, but 1 for k_gemm's MFMA-fragment loads,
    profiles/r03_fetch_calib_v1.txt; pmc_<config>.json records the factor per kernel), or None."""
    path = os.path.join(ROOT, "profiles", f"pmc_{config}.json")
    try:
        with open(path) as fh:
            d = json.load(fh)
        k = d["kernels"][kernel]
        return k["traffic_bytes_per_launch"], os.path.relpath(path, ROOT)
    except (OSError, KeyError, ValueError):
        return None, None


def rocprof_family_avg(kernel, config, flops_per_launch, peak=None):
    """Calls-weighted average duration of `kernel`'s instances in the newest committed
    profiles/r*_<config>_kernel_stats_*.csv and the roofline fraction it gives."""
    import csv
    # r<round>_<config>_kernel_stats_v<n>.csv exactly (not another config's name ending in <config>),
    # newest round, then highest version
    pat = re.compile(rf"r(\d+)_{re.escape(config)}_kernel_stats_v(\d+)\.csv$")
    found = [(int(m.group(1)), int(m.group(2)), p) for p in glob.glob(os.path.join(ROOT, "profiles", "*.csv"))
             for m in [pat.match(os.path.basename(p))] if m]
    paths = [p for _, _, p in sorted(found)]
    if not paths:
        return {}
    tot, n = 0.0, 0
    with open(paths[-1]) as fh:
        for r in csv.DictReader(fh):
            # the plan's GEMM launches: k_gemm, k_gemm_head and k_fwd2 (two forward layers per launch)
            if (f"::{kernel}<" in r["Name"] or f"::{kernel}(" in r["Name"] or f"{kernel}_head<" in r["Name"]
                    or (kernel == "k_gemm" and "::k_fwd2<" in r["Name"])):
                tot += float(r["TotalDurationNs"])
                n += int(r["Calls"])
    if n == 0:
        return {}
    avg_us = tot / n / 1e3
    return {"rocprof_stats": os.path.relpath(paths[-1], ROOT), "rocprof_avg_launch_us": round(avg_us, 3),
            "rocprof_calls": n,
            "rocprof_frac": round(flops_per_launch / (avg_us * 1e-6) / ((peak or FP32_PEAK_TFLOPS) * 1e12), 5)}


def pmc_counter(kernel, config, counter):
    """Mean per-dispatch value of a PMC counter of `kernel` from profiles/pmc_<config>.json."""
    try:
        with open(os.path.join(ROOT, "profiles", f"pmc_{config}.json")) as fh:
            return float(json.load(fh)["kernels"][kernel][counter])
    except (OSError, KeyError, ValueError):
        return None


def roofline(eng, config, n_prof=20, n_replays=20):
    """Roofline of the dominant kernel family (by eager device time).

    Its average launch duration is measured in the real pipeline: a replay of the
    captured update graph in which each launch of the family stores per-workgroup
    s_memrealtime ticks (sacx_time_kernels); a launch lasts from its first workgroup's
    start to its last workgroup's end -- the window rocprofv3 --kernel-trace reports
    for it (profiles/).  HIP events bracket whole graph replays only: an event between
    two graph nodes costs ~4 us of GPU time and would distort the chain.  Must run after
    the timed region (these replays are real updates).  Cross-checks kept in the line:
    the graph time with and without the family (sacx_time_graph) and the eager
    per-stage event times (each includes ~4 us of event overhead)."""
    peak = BF16_PEAK_TFLOPS if CONFIGS[config].get("bf16") else FP32_PEAK_TFLOPS
    info = eng.plan_info()
    ms = eng.profile(n_prof)
    fam = {}
    for i, L in enumerate(info):
        f = fam.setdefault(L["kernel"], dict(ms=0.0, flops=0.0, bytes=0.0, launches=0))
        f["ms"] += ms[i]
        f["flops"] += L["flops"]
        f["bytes"] += L["bytes"]
        f["launches"] += 1
    # the sampler and gather run on the side stream, off the update's critical path
    dom = max((k for k in fam if k not in ("k_rng", "k_gather")), key=lambda k: fam[k]["ms"])
    f = fam[dom]
    G = eng.cfg.graph_steps
    avg_us, us_per_update, n_graph = eng.time_kernels(dom, 3)
    launches = n_graph / G                       # launches per update in the captured graph
    flops_per_launch = f["flops"] / launches     # the plan's family FLOPs per update, folded launches included
    achieved = flops_per_launch / (avg_us * 1e-6) / 1e12
    traffic, src = pmc_traffic(dom, config)
    mfma = pmc_counter(dom, config, "SQ_VALU_MFMA_BUSY_CYCLES")
    t_full = eng.time_graph(n_replays)
    t_wo = eng.time_graph(n_replays, dom)
    rp = rocprof_family_avg(dom, config, flops_per_launch, peak)
    # `achieved` / `frac` come from the committed rocprofv3 --kernel-trace --stats summary of this
    # command (profiles/r<round>_<config>_kernel_stats_v<n>.csv: the family's calls-weighted average
    # duration), so that frac x peak x avg_launch_us reproduces by hand from profiles/; the live
    # per-workgroup stamps of this run are reported beside them as *_live
    avg_rp = rp.get("rocprof_avg_launch_us")
    achieved_rp = flops_per_launch / (avg_rp * 1e-6) / 1e12 if avg_rp else None
    out = {
        "kernel": dom, "bound": "mfma",
        "achieved": round(achieved_rp if avg_rp else achieved, 3), "peak": peak,
        "unit": "TFLOP/s", "frac": round((achieved_rp if avg_rp else achieved) / peak, 5),
        "frac_source": rp.get("rocprof_stats") or "live stamps (no committed rocprof summary)",
        "achieved_live": round(achieved, 3), "frac_live": round(achieved / peak, 5),
        "traffic": traffic, "traffic_source": src,
        # matrix-pipe busy cycles per launch (PMC, summed over the 1,024 SIMDs) over the launch's
        # SIMD-cycles at 2.4 GHz: the counter-side view of `frac`
        "mfma_busy_frac": round(mfma / ((avg_rp or avg_us) * 1e-6 * 2.4e9 * 1024), 5) if mfma else None,
        "avg_launch_us": round(avg_rp if avg_rp else avg_us, 3), "avg_launch_us_live": round(avg_us, 3),
        "launches_per_update": round(launches, 3),
        # per-kernel HBM GB/s and MFMA busy for every kernel (k_gather, k_rng, DW+Adam ...)
        "kernel_table": next((os.path.relpath(p, ROOT) for p in sorted(
            glob.glob(os.path.join(ROOT, "profiles", f"r*_{config}_kernel_table_*.md")))[-1:]), None),
        "flops_per_launch": flops_per_launch,
        "algorithmic_bytes_per_launch": f["bytes"] / launches,
        # the committed rocprofv3 --kernel-trace --stats summary of this command (calls-weighted
        # over every k_gemm instance): its dispatch window includes the end-of-kernel release
        **rp,
        "timing_live": "per-workgroup device timestamps in a replay of the update graph (sacx_time_kernels)",
        "family_us_per_update": round(us_per_update, 3),
        "graph_us_per_update": round(t_full * 1e3, 3),
        "graph_us_per_update_without_family": round(t_wo * 1e3, 3),
        "stage_us_eager_events": {L["name"]: round(float(ms[i]) * 1e3, 2) for i, L in enumerate(info)},
    }
    return out, fam


def host_cpu_info():
    """(os.cpu_count(), cores this process may use, lscpu model name).  On the GPU box
    os.cpu_count() is the whole machine; the usable share is the affinity set capped by the
    cgroup CPU quota (cpu.max) and the box's OMP_NUM_THREADS."""
    total = os.cpu_count() or 1
    usable = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else total
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, p = fh.read().split()[:2]
        if q != "max":
            usable = min(usable, max(1, int(int(q) // int(p))))
    except (OSError, ValueError):
        pass
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if omp > 0:
        usable = min(usable, omp)
    model = None
    try:
        import subprocess
        for ln in subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout.splitlines():
            if ln.lower().startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except Exception:  # pragma: no cover
        pass
    return total, usable, model


def cpu_baseline(cfgd, seconds=10.0):
    """The reference-equivalent CPU path on the host cores (TensorFlow is not installable, so the
    reference itself cannot run): ``oracle/sac_eager_torch.py``, an eager op-by-op PyTorch-CPU
    restatement of ``_update`` with the reference's per-op dispatch structure and Keras Adam
    (SURVEY.md §8d), timed at 1 thread and at every usable core; ``value`` is the faster.  Beside
    it: the vectorised NumPy fp32 oracle (no per-op dispatch: an upper bound on a CPU port), and
    config C1 (SAC-EO: the expert term through two 512x2 world models, plus the per-episode model
    fit amortised at the reference defaults: 5 fit steps per update)."""
    total, usable, model = host_cpu_info()
    q = seconds / 4.0
    eager = {th: _eager_rate(cfgd, q / (2 if usable > 1 else 1), th) for th in sorted({1, usable})}
    best = max(eager, key=lambda t: eager[t][0])
    v, n, el = eager[best][:3]
    npy = {th: _cpu_port_rate(cfgd, q / (2 if usable > 1 else 1), th) for th in sorted({1, usable})}
    nb = max(npy, key=lambda t: npy[t][0])
    c1 = _eager_c1(cfgd, q, best)
    return {"value": round(v, 3), "unit": "gradient-steps/s", "cores": best, "kind": "port",
            "path": "reference-equivalent: eager op-by-op PyTorch-CPU restatement of _update "
                    "(oracle/sac_eager_torch.py; TensorFlow reference not installable)",
            "value_1thread": round(eager[1][0], 3), "value_all_cores": round(eager[usable][0], 3),
            "cores_usable": usable, "os_cpu_count": total, "cpu_model": model,
            "sample": f"{n} eager updates at the bench shapes in {el:.1f}s at {best} thread(s) "
                      f"(also timed at 1 and {usable} threads)",
            "numpy_oracle": {"value": round(npy[nb][0], 3), "cores": nb, "value_1thread": round(npy[1][0], 3),
                             "value_all_cores": round(npy[usable][0], 3),
                             "path": "vectorised NumPy fp32 oracle (oracle/sac_oracle.py), no per-op dispatch"},
            "c1_sac_eo": c1}


def _eager_rate(cfgd, seconds, threads, use_expert=False):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import sac_oracle as O
    import sac_eager_torch as E
    ocfg = O.Config(S=cfgd["S"], A=cfgd["A"], B=cfgd["B"], hidden=cfgd["hidden"], act="relu")
    st = O.init_state(ocfg, seed=1, with_models=use_expert)
    return E.time_updates(st, ocfg, seconds, threads, use_expert=use_expert)


def _eager_c1(cfgd, seconds, threads):
    """Config C1 on the CPU: SAC-EO updates (expert term, 2 world models 512x2, 20 expert rows) and
    model-fit steps (2 x minibatch 200) of the eager restatement; per update the reference also
    runs 5 fit steps at its defaults (1e5 model rows x 10 epochs / 200 per episode of 1,000 steps)."""
    import sac_eager_torch as E
    r, n, el, eng, buf = _eager_rate(cfgd, seconds / 2, threads, use_expert=True)
    f, nf, elf = E.time_model_fit(eng, buf, eng.cfg, seconds / 2)
    return {"updates_per_s": round(r, 3), "fit_steps_per_s": round(f, 3),
            "value": round(1.0 / (1.0 / r + 5.0 / f), 3), "unit": "gradient-steps/s incl. amortised model fit",
            "cores": threads, "sample": f"{n} SAC-EO updates and {nf} model-fit steps (eager PyTorch-CPU)"}


def _cpu_port_rate(cfgd, seconds, threads):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import sac_oracle as O
    try:
        from threadpoolctl import threadpool_limits
        ctx = threadpool_limits(limits=threads)
    except Exception:  # pragma: no cover
        ctx = None
    S, A, B = cfgd["S"], cfgd["A"], cfgd["B"]
    ocfg = O.Config(S=S, A=A, B=B, hidden=cfgd["hidden"], act="relu")
    st = O.init_state(ocfg, seed=1)
    rs = np.random.RandomState(0)
    N = 100_000   # sample of the buffer; gather cost is independent of N
    buf = dict(s=rs.normal(size=(N, S)).astype(np.float32), a=rs.uniform(-1, 1, (N, A)).astype(np.float32),
               sp=rs.normal(size=(N, S)).astype(np.float32), r=rs.normal(size=N).astype(np.float32),
               d=np.zeros(N))
    nrm = O.Normalizers.identity(S, A)
    g = np.random.RandomState(1)
    n = 0
    t0 = time.perf_counter()
    while True:
        R = O.draw_step_randoms(g, N, B, A)
        O.sac_update(st, ocfg, nrm, O.gather(buf, R["idx"]), O.f32_noise(R["noise_t"]),
                     O.f32_noise(R["noise_pi"]), O.f32_noise(R["noise_alpha"]))
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds and n >= 5:
            break
    if ctx is not None:
        ctx.unregister() if hasattr(ctx, "unregister") else None
    return n / el, n, el


def drop_in_loop(eng, cfgd, n=300):
    """The drop-in train loop's rate (algs/SAC_expert.py: one update per env step in the
    reference's order, SAC_expert.py:779-797: a = actor.sample(obs); _update; env.step(a);
    env_data.add): per iteration the behaviour action of one observation comes back to the host
    (B=1), step(1) runs one update, and the transition is appended to the device ring.  The
    action is deterministic, the reference's default behaviour policy (:779, --random_act off).
    act_host queues the next update's sampler draw behind the action kernel, so step(1) replays
    the sampler-less graph (spec_hits counts it)."""
    S, A = cfgd["S"], cfgd["A"]
    rs = np.random.RandomState(0)
    obs = [rs.normal(size=S).astype(np.float32) for _ in range(16)]   # a gym env's host arrays
    r1, d1 = np.zeros(1, np.float32), np.zeros(1, np.float32)
    eng.prepare(1)

    def it(j):
        o, o2 = obs[j % 16], obs[(j + 1) % 16]
        a = eng.act_host(o, deterministic=True)                # host env gets the action
        eng.step(1, num_timesteps=j, ts_increment=1)
        eng.append(o[None], a[None], r1, o2[None], d1)         # the transition, from the host
    for j in range(10):
        it(j)
    eng.sync()
    h0 = eng.spec_hits()
    t0 = time.perf_counter()
    for j in range(n):
        it(j)
    eng.sync()
    el = time.perf_counter() - t0
    return {"updates_per_s": round(n / el, 1), "us_per_iteration": round(el / n * 1e6, 2), "iterations": n,
            "speculative_steps": eng.spec_hits() - h0,
            "iteration": "act(1 host obs, deterministic: the default behaviour policy) -> host action, "
                         "step(1), append(1 host transition)"}


def world_model_legs(eng, cfgd, n_fit=200, n_roll=20):
    """SAC-EO's world-model calls at the reference defaults (rank 0, after the timed
    region): model fitting (A16: 2 models x minibatch 200 per step, SAC_expert.py:519-550)
    and the rollout (F2: --sim_batch_size 10000 over 2 models = 1000 trajectories x
    --sim_horizon 5 per model, mbrl_onpolicy_alg.py:72-100)."""
    import torch
    S, A = cfgd["S"], cfgd["A"]
    mb = eng.cfg.model_batch
    idx = np.random.RandomState(3).randint(cfgd["buffer"], size=(n_fit + 10, 2, mb))
    eng.model_fit(idx[:10])
    eng.sync()
    t0 = time.perf_counter()
    eng.model_fit(idx[10:])
    eng.sync()
    fit_s = (time.perf_counter() - t0) / n_fit
    Hm = 512
    macs = 3 * ((S + A) * Hm + Hm * Hm + Hm * (S + 1)) - (S + A) * Hm      # SURVEY.md §8d model-fit row
    fit_flops = 2.0 * macs * 2 * mb
    s0 = torch.randn(1000, S, device=eng.device)
    eng.rollout(0, s0, 5)
    eng.sync()
    t0 = time.perf_counter()
    for _ in range(n_roll):
        eng.rollout(0, s0, 5)
    eng.sync()
    roll_s = (time.perf_counter() - t0) / n_roll
    return ({"steps_per_s": round(1.0 / fit_s, 1), "us_per_step": round(fit_s * 1e6, 2),
             "tflops": round(fit_flops / fit_s / 1e12, 3), "models": 2, "minibatch": mb, "graph": True},
            {"n_traj": 1000, "horizon": 5, "ms_per_call": round(roll_s * 1e3, 4),
             "transitions_per_s": round(5000 / roll_s, 1), "launches_per_step": 9, "graph": True})


def model_fit_leg(rep, n_fit=512):
    """SAC-EO's world-model fit (A16) at the HalfCheetah shapes of config C1 (the reference's default
    algorithm: 2 world models 512x2, minibatch 200, SAC_expert.py:480-552 / mbrl_onpolicy_alg.py:301-319),
    graph replay of the folded fit chain, timed after the main region on rank 0.  At the reference
    defaults an episode runs ~5,000 fit steps beside its 1,000 updates."""
    cfgd = dict(CONFIGS["hc_eo"], buffer=200_000)
    eng = build_engine(cfgd, rep.seeds(0), device=rep.device)
    mb = eng.cfg.model_batch
    idx = np.random.RandomState(3).randint(cfgd["buffer"], size=(n_fit + 64, 2, mb))
    eng.model_fit(idx[:64])
    eng.sync()
    t0 = time.perf_counter()
    eng.model_fit(idx[64:])
    eng.sync()
    us = (time.perf_counter() - t0) / n_fit * 1e6
    S, A, Hm = cfgd["S"], cfgd["A"], 512
    macs = 3 * ((S + A) * Hm + Hm * Hm + Hm * (S + 1)) - (S + A) * Hm      # SURVEY.md section 8d model-fit row
    flops = 2.0 * macs * 2 * mb
    launches = eng.model_plan_info()
    eng.close()
    out = {"config": "HalfCheetah-shaped SAC-EO world-model fit: 2 models 512x2, minibatch 200 (config C1 shapes)",
           "steps": n_fit, "us_per_step": round(us, 2), "steps_per_s": round(1e6 / us, 1),
           "flops_per_step": flops, "achieved_tflops": round(flops / us / 1e6, 3),
           "frac_fp32_peak": round(flops / us / 1e6 / FP32_PEAK_TFLOPS, 5), "graph": True}
    gemms = [L for L in launches if L["kernel"] == "k_gemm"]
    out["launches_per_step"] = len(launches)
    out["launches"] = [L["name"] for L in launches]
    out["us_per_launch"] = round(us / max(1, len(launches)), 3)
    # the committed rocprofv3 --kernel-trace --stats summary of the fit (tools/gpu_run.sh mprof)
    out.update(rocprof_family_avg("k_gemm", "mfit_hc", sum(L["flops"] for L in gemms) / max(1, len(gemms))))
    return out


def replica_seeds(rep, k):
    """The reference-style seeds of this replica's k learners: run indices rank*k .. rank*k+k-1
    of derive_seeds (sac_eo/train.py:108-118), one dict per learner."""
    from sac_eo.common.seeding import derive_seeds
    if k <= 1:
        return rep.seeds(0)
    ds = derive_seeds(0, runs=rep.world_size * k)
    return [{n: int(v[rep.rank * k + j]) for n, v in ds.items()} for j in range(k)]


def packed_leg(cfgd, config, rep, k, steps, with_roofline):
    """K independent learners packed into one handle per GPU (cfg.seeds = K: every launch of the
    update graph runs all K, grid z = seed): whole-job updates/s over all seeds and GPUs, timed
    like the main region (barrier + synchronize, max over ranks).  The k_gemm roofline of the
    packed chain counts the K seeds' FLOPs per launch."""
    eng = build_engine(cfgd, replica_seeds(rep, k), device=rep.device)
    eng.step(256)
    # a steady-state figure whatever --steps says: at least 4 full 128-update graphs (a 20-step
    # region is two graph launches and two sampler ramps, not the packed chain's rate)
    steps = max(steps, 512)
    cap_s = eng.prepare(steps)          # every graph step(steps) replays, instantiated untimed
    eng.sync()
    rep.barrier()
    t0 = time.perf_counter()
    eng.step(steps)
    eng.sync()
    t1 = time.perf_counter()
    rep.barrier()
    el = rep.max_over_ranks(t1 - t0)
    finite = True
    for j in range(k):
        eng.select_seed(j)
        finite = finite and bool(np.all(np.isfinite(eng.stats(1)[0])))
    eng.select_seed(0)
    out = {"seeds_per_gpu": k, "value": round(steps * k * rep.world_size / el, 2), "unit": "gradient-steps/s",
           "per_seed": round(steps / el, 2), "ms_per_round": round(el / steps * 1e3, 5), "steps": steps,
           "finite_stats": finite, "graph_prepare_s": round(cap_s, 4),
           "note": "independent learners (the reference's --runs) packed into one handle per GPU"}
    if with_roofline:
        peak = BF16_PEAK_TFLOPS if cfgd.get("bf16") else FP32_PEAK_TFLOPS
        info = eng.plan_info()
        flops = sum(L["flops"] for L in info if L["kernel"] == "k_gemm")     # one seed, per update
        avg_us, _, n_graph = eng.time_kernels("k_gemm", 3)
        fpl = k * flops / (n_graph / eng.cfg.graph_steps)
        out["roofline"] = {"kernel": "k_gemm", "bound": "mfma", "achieved": round(fpl / (avg_us * 1e-6) / 1e12, 3),
                           "peak": peak, "unit": "TFLOP/s",
                           "frac": round(fpl / (avg_us * 1e-6) / 1e12 / peak, 5), "avg_launch_us": round(avg_us, 3),
                           "flops_per_launch": fpl,
                           "timing": "per-workgroup device timestamps in a replay of the packed update graph"}
    eng.close()
    return out


def _ranks_cmd(n, argv):
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)


def spawn_ranks(n):
    """Runs this script as n ranks under torch.distributed.run (127.0.0.1 rendezvous) in a
    child process; returns its exit status.  The parent never initialises the GPU."""
    import subprocess
    return subprocess.call(_ranks_cmd(n, sys.argv[1:]))


DP_CHECK_UPDATES = 64


def dp_check(cfgd, rep, n_check=DP_CHECK_UPDATES, n_time=512):
    """Config C4 over RCCL (``--mode dpcheck``, run by the N > 1 bench as a child launch): one
    learner over the ws ranks of a fresh RCCL group (sacx_dp_init: ncclAllReduce of the critic,
    actor and alpha gradients inside the captured update graph), each rank sampling B / ws rows of
    its own replica of the replay ring (identical rows and initial weights on every rank) from its
    own stream.
      1. ``n_check`` updates from host-drawn randoms (SACX_STEP_EXTERNAL_RANDOMS, each rank its own
         RandomState): every rank's parameters, targets and Adam moments must be bit-identical
         (sha256 over the arena's PARAM / STATE prefix, gathered), and equal, within 1e-4 relative
         to each tensor's max, a single learner's updates on the concatenated B-row batches (rank 0
         replays them with the gathered indices and noise);
      2. ``n_time`` graph-replayed updates with the device samplers: updates/s of the one learner.
    Returns rank 0's result dict (None elsewhere)."""
    import hashlib
    import torch
    from sac_eo.common.seeding import derive_seeds
    from sac_eo.engine import Engine
    ws, rank, device = rep.world_size, rep.rank, rep.device
    S, A, B = cfgd["S"], cfgd["A"], cfgd["B"]
    if cfgd["use_expert"] or B % ws:
        raise SystemExit("dpcheck: plain SAC configs with batch divisible by the GPU count")
    Bl, N = B // ws, cfgd["buffer"]
    shared = {k: int(v[0]) for k, v in derive_seeds(0, runs=1).items()}   # rows and weights of run 0
    comm_ws = rep.dist.get_world_size() if rep.dist is not None else 1
    uid = rep.broadcast_bytes(Engine.dp_unique_id() if rank == 0 else None)
    eng = build_engine(cfgd, shared, device, dp=(uid, ws, rank), batch=Bl, weight_seed=shared["setup"])
    rs = np.random.RandomState(7000 + rank)
    idx_all, nz_all = [], []
    for t in range(n_check):
        idx = rs.randint(N, size=Bl)                          # buffers.py:136 on this rank's stream
        nz = rs.normal(size=(3, Bl, A))                       # target, policy, alpha evaluate()
        eng.v["slot0.idx"][0].copy_(torch.from_numpy(idx.astype(np.int32)))
        eng.v["slot0.noise"][0][:3 * Bl * A].copy_(torch.from_numpy(nz.astype(np.float32).ravel()))
        eng.step(1, num_timesteps=t, ts_increment=1, external=True)
        idx_all.append(idx)
        nz_all.append(nz)
    eng.sync()
    end = eng.segments["grad"]["offset"]                      # params, adam_m, adam_v (targets included)
    digest = hashlib.sha256(eng.arena[:end].cpu().numpy().tobytes()).hexdigest()
    mine = dict(digest=digest, idx=np.stack(idx_all), nz=np.stack(nz_all))
    allr = [None] * ws
    rep.dist.all_gather_object(allr, mine)
    identical = all(r["digest"] == allr[0]["digest"] for r in allr)
    dev_nets = {n: eng.get_net(n) for n in ("actor", "q0", "q1", "t0", "t1")}
    dev_alpha = eng.alpha()
    # timed: the device samplers, graph replays (every rank the same global update)
    eng.step(16, num_timesteps=n_check, ts_increment=1)
    eng.prepare(n_time)
    rep.barrier()
    t0 = time.perf_counter()
    eng.step(n_time, num_timesteps=n_check + 16, ts_increment=1)
    eng.sync()
    el = rep.max_over_ranks(time.perf_counter() - t0)
    eng.close()
    rep.barrier()
    if rank != 0:
        return None
    # the single learner on the concatenated batches (rank order: ranks' rows, then per draw)
    one = build_engine(cfgd, shared, device, batch=B, weight_seed=shared["setup"])
    for t in range(n_check):
        idx = np.concatenate([r["idx"][t] for r in allr])
        nz = np.concatenate([r["nz"][t] for r in allr], axis=1)      # [3, B, A]
        one.v["slot0.idx"][0].copy_(torch.from_numpy(idx.astype(np.int32)))
        one.v["slot0.noise"][0][:3 * B * A].copy_(torch.from_numpy(nz.astype(np.float32).ravel()))
        one.step(1, num_timesteps=t, ts_increment=1, external=True)
    one.sync()
    worst = 0.0
    for n, ws_dev in dev_nets.items():
        for a_, b_ in zip(ws_dev, one.get_net(n)):
            worst = max(worst, float(np.max(np.abs(a_ - b_)) / max(float(np.max(np.abs(b_))), 1e-30)))
    d_alpha = abs(dev_alpha - one.alpha()) / max(abs(one.alpha()), 1e-5)
    one.close()
    return {"ranks": ws, "rccl_world_size": comm_ws, "backend": rep.backend, "local_batch": Bl,
            "checked_updates": n_check, "dp_ranks_identical": identical,
            "vs_single_learner_max_rel_err": worst, "alpha_rel_err": d_alpha,
            "matches_single_learner": bool(worst < 1e-4 and d_alpha < 1e-4),
            "timed_updates": n_time, "updates_per_s": round(n_time / el, 2),
            "ms_per_update": round(el / n_time * 1e3, 4),
            "note": "one learner over the ranks (strong scaling); 3 RCCL all-reduces per update inside the graph"}


def run_dp_child(ws, config, timeout=180):
    """The C4 leg of an N > 1 bench: a fresh ws-rank launch of ``--mode dpcheck`` (its own RCCL
    group), started by rank 0 after every replica rank has released its GPU; a hang or failure of
    the leg costs only its own entry, never the replicas line."""
    import subprocess
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK",
                        "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID") and not k.startswith("TORCHELASTIC")}
    cmd = _ranks_cmd(ws, ["--mode", "dpcheck", "--gpus", str(ws), "--config", config])
    try:
        out = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)
    except subprocess.TimeoutExpired:
        return {"ranks": ws, "error": f"timed out after {timeout} s"}
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    if out.returncode != 0 or not lines:
        return {"ranks": ws, "error": f"exit {out.returncode}", "stderr_tail": out.stderr[-800:]}
    return json.loads(lines[-1]).get("dp_c4")


def plan_only(args):
    """The launch plan without a GPU: each rank joins a gloo group and reports its rank, the
    world size the group sees and its learners' seeds (replica_seeds); rank 0 prints one JSON
    line with every rank's entry (tests/test_replicas.py checks it for --gpus 2)."""
    from sac_eo.common.replicas import init_replica
    rep = init_replica(backend="gloo", use_cuda=False)
    mine = {"rank": rep.rank, "world_size": rep.world_size, "seeds": replica_seeds(rep, args.seeds_per_gpu),
            "group_world_size": rep.dist.get_world_size() if rep.dist is not None else 1,
            "backend_on_gpus": "nccl (RCCL)"}
    if rep.dist is not None:
        allr = [None] * rep.world_size
        rep.dist.all_gather_object(allr, mine)
    else:
        allr = [mine]
    if rep.rank == 0:
        # the N > 1 line's C4 leg: a fresh launch of --mode dpcheck over all the ranks' GPUs
        leg = None if args.gpus < 2 else {"ranks": args.gpus, "mode": "dpcheck",
                                          "checked_updates": DP_CHECK_UPDATES,
                                          "fields": ["dp_ranks_identical", "vs_single_learner_max_rel_err",
                                                     "rccl_world_size", "updates_per_s"]}
        print(json.dumps({"plan_only": True, "n_gpus": args.gpus, "ranks": allr, "dp_c4_leg": leg,
                          "line_fields_n_gt_1": ["rank_times_s", "group_world_size", "dp_c4"]}), flush=True)
    rep.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--config", default="hc", choices=sorted(CONFIGS))
    ap.add_argument("--cpu-seconds", type=float, default=16.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--mode", default="replicas", choices=["replicas", "dp", "dpcheck"],
                    help="replicas: one independent learner per GPU (the metric); dp: one learner, "
                         "global batch split over the GPUs, gradients all-reduced by RCCL (config C4)")
    ap.add_argument("--seeds-per-gpu", type=int, default=1,
                    help="independent learners packed into each GPU's handle for the timed region "
                         "(one launch chain, grid z = seed); value counts the updates of every seed")
    ap.add_argument("--packed-leg", type=int, default=-1,
                    help="after the timed region, also time K packed seeds per GPU and report them as "
                         "packed_seeds (default 8 for hc, 4 for the Humanoid configs; 0 = off)")
    ap.add_argument("--no-dp-leg", action="store_true",
                    help="N > 1: skip the C4 data-parallel RCCL leg (a child launch of --mode dpcheck)")
    ap.add_argument("--plan-only", action="store_true",
                    help="no GPU: every rank joins a gloo group and prints its rank and seeds (launch check)")
    args = ap.parse_args()

    # --gpus N without a torch.distributed.run environment: relaunch as N ranks (one per GPU)
    # through torch.distributed.run, from this process before anything touches the GPU, and
    # exit with the launcher's status.  Under the launcher WORLD_SIZE must equal --gpus.
    ws_env = os.environ.get("WORLD_SIZE")
    if ws_env is None and args.gpus > 1:
        raise SystemExit(spawn_ranks(args.gpus))
    if int(ws_env or 1) != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={ws_env}")
    if args.plan_only:
        plan_only(args)
        return

    import torch
    from sac_eo.common.replicas import init_replica
    rep = init_replica()                      # one learner per GPU, RCCL only for barrier / max time
    ws, rank, device = rep.world_size, rep.rank, rep.device
    cfgd = CONFIGS[args.config]
    if args.mode == "dpcheck":
        res = dp_check(cfgd, rep)
        if rank == 0:
            print(json.dumps({"dp_c4": res}), flush=True)
        rep.close()
        return
    dp = args.mode == "dp"
    if dp:
        from sac_eo.engine import Engine
        from sac_eo.common.seeding import derive_seeds
        if cfgd["use_expert"] or cfgd["B"] % ws:
            raise SystemExit("dp mode: plain SAC configs with batch divisible by the GPU count")
        uid = rep.broadcast_bytes(Engine.dp_unique_id() if rank == 0 else None)
        eng = build_engine(cfgd, rep.seeds(0), device=device, dp=(uid, ws, rank), batch=cfgd["B"] // ws,
                           weight_seed=int(derive_seeds(0, runs=1)["setup"][0]))
    else:
        eng = build_engine(cfgd, replica_seeds(rep, args.seeds_per_gpu), device=device)
    K = 1 if dp else max(1, args.seeds_per_gpu)
    barrier = rep.barrier

    eng.step(args.warmup, num_timesteps=0, ts_increment=1)
    # capture + instantiate + upload every graph the timed step(steps) replays (untimed;
    # reported as graph_prepare_s): the timed region launches cached graphs only
    cap_s = eng.prepare(args.steps)
    eng.sync()
    barrier()
    t0 = time.perf_counter()
    eng.step(args.steps, num_timesteps=args.warmup, ts_increment=1)
    eng.sync()
    t1 = time.perf_counter()
    barrier()
    el = rep.max_over_ranks(t1 - t0)
    rank_times = [t1 - t0]
    if rep.dist is not None:                  # every rank's own timed region
        rank_times = [None] * ws
        rep.dist.all_gather_object(rank_times, t1 - t0)
    stats = eng.stats(1)[0]
    finite = bool(np.all(np.isfinite(stats)))
    value = args.steps * (1 if dp else ws * K) / el     # dp: every rank runs the same global update
    # secondary legs on rank 0, after the timed region; the roofline leg last (its ablated
    # graph replay leaves the learner's state meaningless)
    loop = None
    if rank == 0 and K == 1 and not dp and not args.no_roofline:
        loop = drop_in_loop(eng, cfgd)
    fit = roll = None
    if rank == 0 and cfgd["use_expert"] and K == 1:
        fit, roll = world_model_legs(eng, cfgd)
    mfit = None
    if rank == 0 and not args.no_roofline and not dp and K == 1 and args.config == "hc":
        mfit = model_fit_leg(rep)
    roof = None
    if rank == 0 and not args.no_roofline and not dp:
        roof, _ = roofline(eng, args.config)
    packed = None
    nleg = args.packed_leg if args.packed_leg >= 0 else (8 if args.config == "hc" else 4)
    if not dp and K == 1 and nleg > 1:
        eng.close()
        eng = None
        packed = packed_leg(cfgd, args.config, rep, nleg, min(args.steps, 1024), rank == 0 and not args.no_roofline)
    cpu = None
    if rank == 0 and ws == 1 and not args.no_cpu_baseline and not dp:
        cpu = cpu_baseline(cfgd, args.cpu_seconds)
    group_ws = rep.dist.get_world_size() if rep.dist is not None else 1
    dpres = None
    if ws > 1 and not dp and not args.no_dp_leg:
        # config C4 over RCCL: every replica rank releases its GPU, rank 0 starts the ws-rank
        # dpcheck launch (its own group), waits for it (bounded), then prints the line
        import torch
        if eng is not None:
            eng.close()
            eng = None
        rep.barrier()
        rep.close()
        torch.cuda.empty_cache()
        if rank != 0:
            return
        if torch.cuda.device_count() < ws:
            dpres = {"ranks": ws, "skipped": f"{torch.cuda.device_count()} visible GPUs for {ws} ranks "
                                               "(RCCL needs one GPU per rank)"}
        else:
            dpres = run_dp_child(ws, args.config)
    if rank == 0:
        line = {
            "metric": ("SAC" + ("-EO" if cfgd["use_expert"] else "") + " gradient-steps/sec ("
                       + ("" if cfgd["S"] == 17 else "Humanoid-shaped, ")
                       + f"batch={cfgd['B']}, 256x2 MLP)"),
            "value": round(value, 2), "unit": "gradient-steps/s", "n_gpus": ws, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 5), "higher_is_better": True,
            "scaling": "strong" if dp else "weak", "vs_baseline": None,
            "dtype": "bf16 (MFMA operands), f32 accumulate" if cfgd.get("bf16") else "f32",
            "data": ("synthetic (" + ("HalfCheetah" if cfgd["S"] == 17 else "Humanoid")
                     + "-shaped replay rows generated on device; random orthogonal init)"),
            "config": {"workload": cfgd["workload"], "obs_dim": cfgd["S"], "act_dim": cfgd["A"],
                       "batch": cfgd["B"], "hidden": list(cfgd["hidden"]), "buffer_rows": cfgd["buffer"],
                       "parallelism": (f"dp{ws}: one learner, batch {cfgd['B'] // ws} per GPU, 3 RCCL all-reduces "
                                       "per update (critic, actor, alpha gradients)") if dp else
                                      (f"replicas x{ws} (independent seeds, no collective)" if K == 1 else
                                       f"replicas x{ws} x {K} packed seeds per GPU (independent seeds, no collective)"),
                       "seeds_per_gpu": K,
                       "sampler": "NumPy-legacy MT19937 stream on device (bit-exact indices)"},
            "finite_stats": finite, "graph_prepare_s": round(cap_s, 4),
            "last_stats": {k: float(v) for k, v in zip(
                ["q1_loss", "q2_loss", "p_loss", "alpha_loss", "alpha", "mse_loss", "nlp_mean", "step"], stats)},
            "roofline": roof, "cpu_baseline": cpu,
        }
        if ws > 1:
            line["group_world_size"] = group_ws            # torch.distributed group the ranks joined
            line["process_group_backend"] = rep.backend
            line["rank_times_s"] = [round(float(x), 6) for x in rank_times]
            line["dp_c4"] = dpres
        if fit is not None:
            line["model_fit"], line["rollout"] = fit, roll
        if mfit is not None:
            line["model_fit_c1"] = mfit
        if loop is not None:
            line["drop_in_loop"] = loop
        if packed is not None:
            line["packed_seeds"] = packed
        print(json.dumps(line), flush=True)
    if eng is not None:
        eng.close()
    rep.close()


if __name__ == "__main__":
    main()
