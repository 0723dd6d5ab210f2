set -u
mkdir -p gpurun_out/pkab
for r in 1 2; do
for e in X=1 SACX_FOLD_HBW=0 SACX_HEAD_PART=0 "SACX_FOLD_HBW=0 SACX_HEAD_PART=0"; do
  env $e timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --seeds-per-gpu 8 --steps 1024 --warmup 128 > gpurun_out/pkab/out.log 2>&1 || exit 1
  echo "$r [$e] $(python -c "import json,sys; [print(json.loads(l)['value']) for l in open(sys.argv[1]) if l.startswith('{')]" gpurun_out/pkab/out.log)"
done; done
