set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for s in 1 0 1 0; do
  SACX_SPEC=$s timeout -k 10 200 python tools/dropin_parts.py > gpurun_out/dropin_spec$s.log 2>&1 || exit $?
  echo "SPEC=$s"; tail -2 gpurun_out/dropin_spec$s.log
done
timeout -k 10 300 python bench.py --config humanoid_bf16 --no-cpu-baseline --packed-leg 0 > gpurun_out/hum_bf16.log 2>&1 || exit $?
tail -c 600 gpurun_out/hum_bf16.log
