set -u
cd "${GRAFT_REPO_ROOT}"
export SACX_MFUSE=2
for r in 1 2; do
  for v in A B; do
    if [ $v = B ]; then export SACX_LIBPATH=$PWD/tools/libvar/libsacx_dwns4.so; else unset SACX_LIBPATH; fi
    echo "== $v$r"
    timeout -k 10 200 python tools/model_fit_time.py hc_eo 512 2>&1 | grep graph | tail -1 || exit 1
    timeout -k 10 200 python tools/model_fit_time.py humanoid_eo 256 2>&1 | grep graph | tail -1 || exit 1
    timeout -k 10 300 python bench.py --config humanoid_sac --steps 1000 --warmup 100 --no-cpu-baseline --no-roofline --packed-leg 0 2>&1 | grep -o '"value": [0-9.]*' || exit 1
  done
done
