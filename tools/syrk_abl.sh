set -o pipefail
mkdir -p gpurun_out/sa
for v in 0 1 2 4 8 3 5 7 15; do
  SNK_SYRK_DBG=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras --d-snapshots 0 > gpurun_out/sa/b$v.json 2>gpurun_out/sa/e$v.log || exit 2
  python -c "import json;d=json.load(open('gpurun_out/sa/b$v.json'));print('$v', round(d['d_build']['phase_ms']['conv_gram'],1))"
done
