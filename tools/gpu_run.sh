#!/bin/bash
# One gpurun call = a list of named steps, run in order; stops at the first failing step (a test
# failure too: nothing after it is trusted).  Logs under gpurun_out/${TAG:-run}/.
#   bash tools/gpu_run.sh tests [pytest selectors, comma-separated] | smoke | bench[=<bench args>]
#                         | driver | mfit | humanoid | prof=<config> | pmc=<config> | ktime=<config> ...
# e.g. bash tools/gpu_run.sh tests smoke bench "bench=--config hc_eo --no-cpu-baseline" prof=hc
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-run}
mkdir -p "$OUT"
export TMPDIR=/tmp
n=0
value() { grep -o '"value": [0-9.]*' "$1" | head -1; }
for step in "$@"; do
  n=$((n + 1))
  name=${step%%=*}; arg=""; [ "$name" != "$step" ] && arg=${step#*=}
  log=$OUT/$n-$name.log
  case $name in
    tests)
      # tests=<comma-separated paths / options>[|<-k expression, spaces allowed>]
      sel=${arg:-tests}; kx=""
      case $sel in *"|"*) kx=${sel#*|}; sel=${sel%%|*} ;; esac
      if [ -n "$kx" ]; then
        timeout -k 10 1100 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
            ${sel//,/ } -k "$kx" > "$log" 2>&1
      else
        timeout -k 10 1100 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
            ${sel//,/ } > "$log" 2>&1
      fi
      rc=$?; echo "[$n tests] rc=$rc $(tail -n 1 "$log")" ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$log" 2>&1
      rc=$?; echo "[$n smoke] rc=$rc $(tail -n 1 "$log")" ;;
    bench)
      timeout -k 10 500 python bench.py $arg > "$log" 2>&1
      rc=$?; echo "[$n bench $arg] rc=$rc $(value "$log")" ;;
    driver)     # the driver's own command
      timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > "$log" 2>&1
      rc=$?; echo "[$n driver] rc=$rc $(value "$log")" ;;
    mfit)       # world-model fit (A16) at HC and Humanoid shapes
      { timeout -k 10 200 python tools/model_fit_time.py hc_eo 512 && \
        timeout -k 10 200 python tools/model_fit_time.py humanoid_eo 256; } > "$log" 2>&1
      rc=$?; echo "[$n mfit] rc=$rc"; cat "$log" ;;
    driverenv)  # the driver's command under one extra environment setting: driverenv=VAR=VALUE
      env "$arg" timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > "$log" 2>&1
      rc=$?; echo "[$n driverenv $arg] rc=$rc $(value "$log")" ;;
    overheadenv)  # step-overhead table under one extra environment setting
      env "$arg" timeout -k 10 200 python tools/step_overhead.py > "$log" 2>&1
      rc=$?; echo "[$n overheadenv $arg] rc=$rc"; grep -E "n=  20 launch|fit:" "$log" ;;
    n2shared)   # bench --gpus 2 with both ranks on the one visible GPU (gloo replicas; the C4 leg skips)
      SACX_SHARE_DEVICE=1 SACX_REPLICA_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 400 --warmup 50 \
          --no-cpu-baseline > "$log" 2>&1
      rc=$?; echo "[$n n2shared] rc=$rc $(value "$log")"; grep -o '"dp_c4": {[^}]*}' "$log" || true ;;
    cfgenv)     # bench of config C under one extra environment setting: cfgenv=C:VAR=VALUE (VAR=VALUE may be -)
      cfg=${arg%%:*}; ev=${arg#*:}
      if [ "$ev" = "-" ]; then ev="SACX_NOP=1"; fi
      env $ev timeout -k 10 300 python bench.py --config $cfg --steps 1000 --warmup 100 --no-cpu-baseline > "$log" 2>&1
      rc=$?; echo "[$n cfgenv $arg] rc=$rc $(value "$log")" ;;
    mfitv)      # the fit timing with a variant library: mfitv=<tools/libvar name>
      { SACX_LIBPATH=$PWD/tools/libvar/libsacx_$arg.so timeout -k 10 200 python tools/model_fit_time.py hc_eo 512 && \
        SACX_LIBPATH=$PWD/tools/libvar/libsacx_$arg.so timeout -k 10 200 python tools/model_fit_time.py humanoid_eo 256; } > "$log" 2>&1
      rc=$?; echo "[$n mfitv $arg] rc=$rc"; grep graph "$log" ;;
    mfitenv)    # the HC / Humanoid fit timing under one extra environment setting: mfitenv=VAR=VALUE
      { env "$arg" timeout -k 10 200 python tools/model_fit_time.py hc_eo 512 && \
        env "$arg" timeout -k 10 200 python tools/model_fit_time.py humanoid_eo 256; } > "$log" 2>&1
      rc=$?; echo "[$n mfitenv $arg] rc=$rc"; grep graph "$log" ;;
    mtrace)     # kernel trace of the model fit of config $arg: one step's launches, durations, gaps
      cfg=${arg:-hc_eo}
      timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$PWD/$OUT/mtrace_$cfg" -o m \
          -- python tools/model_fit_time.py $cfg 128 > "$log" 2>&1
      rc=$?
      if [ $rc -eq 0 ]; then
        f=$(find "$OUT/mtrace_$cfg" -name "*kernel_trace.csv" | head -1)
        python tools/trace_view.py "$f" 24 "k_mgather,k_gemm<0, 1, 6,k_gemm<0, 0, 6" > "$OUT/$n-mtrace_$cfg.txt" 2>&1; cat "$OUT/$n-mtrace_$cfg.txt"
      fi
      echo "[$n mtrace $cfg] rc=$rc" ;;
    mktime)     # per-launch workgroup timing of the fit (eager steps, SACX_MFIT_KTIME): mktime=<config>
      timeout -k 10 200 python tools/mfit_ktime.py ${arg:-hc_eo} > "$log" 2>&1
      rc=$?; echo "[$n mktime ${arg:-hc_eo}] rc=$rc"; cat "$log" | grep -v amdgpu.ids ;;
    mktimev)    # mktime with a variant library: mktimev=<config>:<tools/libvar name>
      cfg=${arg%%:*}; var=${arg#*:}
      SACX_LIBPATH=$PWD/tools/libvar/libsacx_$var.so timeout -k 10 200 python tools/mfit_ktime.py $cfg > "$log" 2>&1
      rc=$?; echo "[$n mktimev $arg] rc=$rc"; cat "$log" | grep -v amdgpu.ids ;;
    mprof)      # rocprofv3 kernel-trace stats of the HC model fit (graph replay only) -> profiles r*_mfit_hc_kernel_stats
      MFT_GRAPH_ONLY=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/mprof" -o m \
          -- python tools/model_fit_time.py hc_eo 2048 > "$log" 2>&1
      rc=$?; echo "[$n mprof] rc=$rc $(grep graph "$log")" ;;
    humanoid)
      rc=0
      for c in humanoid_sac humanoid_bf16 humanoid_eo; do
        timeout -k 10 300 python bench.py --config $c --steps 1000 --warmup 100 --no-cpu-baseline > "$OUT/$n-$c.log" 2>&1
        rc=$?; echo "[$n $c] rc=$rc $(value "$OUT/$n-$c.log")"; [ $rc -eq 0 ] || break
      done ;;
    prof)       # rocprofv3 kernel-trace stats of the one-seed bench of config $arg
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/prof_${arg:-hc}" -o s \
          -- python bench.py --config "${arg:-hc}" --steps 2000 --warmup 200 --no-cpu-baseline --no-roofline --packed-leg 0 > "$log" 2>&1
      rc=$?; echo "[$n prof ${arg:-hc}] rc=$rc $(value "$log")" ;;
    profenv)    # prof (hc) under one extra environment setting: profenv=VAR=VALUE
      env "$arg" timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/prof_env_$n" -o s \
          -- python bench.py --config hc --steps 2000 --warmup 200 --no-cpu-baseline --no-roofline --packed-leg 0 > "$log" 2>&1
      rc=$?; echo "[$n profenv $arg] rc=$rc $(value "$log")" ;;
    pmc)
      CONFIG=${arg:-hc} bash tools/gpu_pmc.sh > "$log" 2>&1
      rc=$?; echo "[$n pmc ${arg:-hc}] rc=$rc"; tail -n 3 "$log" ;;
    overhead)   # fixed cost of one step(n) call (sampler start-up, alpha tail, launch + wake-up)
      timeout -k 10 200 python tools/step_overhead.py $arg > "$log" 2>&1
      rc=$?; echo "[$n overhead] rc=$rc"; cat "$log" ;;
    mtbench)    # twist-only MT19937 variants (tools/mt_bench.hip, built on the CPU side)
      timeout -k 10 120 ./tools/mt_bench > "$log" 2>&1
      rc=$?; echo "[$n mtbench] rc=$rc"; cat "$log" ;;
    rngbench)
      timeout -k 10 120 ./tools/rng_bench > "$log" 2>&1
      rc=$?; echo "[$n rngbench] rc=$rc"; cat "$log" ;;
    rngenv)     # rng_bench's segmented Humanoid cases under extra environment settings: rngenv=VAR=VALUE[ VAR=VALUE]
      env $arg timeout -k 10 120 ./tools/rng_bench "humanoid seg" > "$log" 2>&1
      rc=$?; echo "[$n rngenv $arg] rc=$rc"; grep 'us/update\|emit per' "$log" ;;
    rngprof)    # rocprofv3 kernel-trace (+ stats) of the rng_bench configurations matching $arg
      timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/rngprof_$n" -o r \
          -- ./tools/rng_bench "$arg" > "$log" 2>&1
      rc=$?; echo "[$n rngprof $arg] rc=$rc"; tail -n 4 "$log" ;;
    ktimev)     # ktime with a variant library: ktimev=<config>:<tools/libvar name>
      cfg=${arg%%:*}; var=${arg#*:}
      SACX_LIBPATH=$PWD/tools/libvar/libsacx_$var.so timeout -k 10 200 python tools/ktime_dump.py "$cfg" > "$log" 2>&1
      rc=$?; echo "[$n ktimev $arg] rc=$rc $(tail -n 1 "$log")" ;;
    ktimeenv)   # ktime (hc) under one extra environment setting: ktimeenv=VAR=VALUE
      env "$arg" timeout -k 10 200 python tools/ktime_dump.py hc > "$log" 2>&1
      rc=$?; echo "[$n ktimeenv $arg] rc=$rc $(tail -n 1 "$log")" ;;
    ktimecfgenv)  # ktime of config C under one extra environment setting: ktimecfgenv=C:VAR=VALUE
      cfg=${arg%%:*}; ev=${arg#*:}
      env "$ev" timeout -k 10 200 python tools/ktime_dump.py "$cfg" > "$log" 2>&1
      rc=$?; echo "[$n ktimecfgenv $arg] rc=$rc $(tail -n 1 "$log")" ;;
    benchenv)   # the 2,000-update bench under one extra environment setting: benchenv=VAR=VALUE
      env "$arg" timeout -k 10 300 python bench.py --steps 2000 --warmup 200 --no-cpu-baseline > "$log" 2>&1
      rc=$?; echo "[$n benchenv $arg] rc=$rc $(value "$log")" ;;
    benchv)     # the 2,000-update HC bench with a variant library: benchv=<tools/libvar name>
      SACX_LIBPATH=$PWD/tools/libvar/libsacx_$arg.so timeout -k 10 300 python bench.py --steps 2000 --warmup 200 --no-cpu-baseline > "$log" 2>&1
      rc=$?; echo "[$n benchv $arg] rc=$rc $(value "$log")" ;;
    dropin)     # host time per drop-in iteration: dropin[=<tools/libvar name>]
      if [ -n "$arg" ]; then lp=$PWD/tools/libvar/libsacx_$arg.so; else lp=$PWD/sac-expert_amd/lib/libsacx.so; fi
      SACX_LIBPATH=$lp timeout -k 10 200 python tools/dropin_trace.py host > "$log" 2>&1
      rc=$?; echo "[$n dropin $arg] rc=$rc $(tail -n 1 "$log")" ;;
    dropinenv)  # dropin under one extra environment setting: dropinenv=VAR=VALUE
      env "$arg" timeout -k 10 200 python tools/dropin_trace.py host > "$log" 2>&1
      rc=$?; echo "[$n dropinenv $arg] rc=$rc $(tail -n 1 "$log")" ;;
    dropintr)   # kernel trace of the drop-in loop (tools/dropin_trace.py), optional env: dropintr=VAR=VALUE
      ev=${arg:-SACX_NONE=0}
      env "$ev" timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$PWD/$OUT/dtr$n" -o d \
          -- python tools/dropin_trace.py run > "$log" 2>&1 && python tools/dropin_trace.py "$OUT/dtr$n" >> "$log" 2>&1
      rc=$?; echo "[$n dropintr $arg] rc=$rc"; grep -A3 "iterations:" "$log" ;;
    runs)       # sac_eo.train --runs K serial vs lock-step packed: runs=<K>:<alg>:<steps>[:VAR=VALUE]
      IFS=: read -r rk ralg rsteps renv <<< "$arg"
      env "${renv:-SACX_NONE=0}" timeout -k 10 400 python tools/packed_runs_time.py "$rk" "$ralg" "$rsteps" 2 > "$log" 2>&1
      rc=$?; echo "[$n runs $arg] rc=$rc"; grep -E "^(serial|packed|pool)" "$log" ;;
    ktime)
      timeout -k 10 200 python tools/ktime_dump.py "${arg:-hc}" > "$log" 2>&1
      rc=$?; echo "[$n ktime ${arg:-hc}] rc=$rc $(tail -n 1 "$log")" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  [ $rc -eq 0 ] || { tail -n 30 "$log"; exit $rc; }
done
