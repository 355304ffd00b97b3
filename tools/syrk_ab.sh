set -o pipefail
mkdir -p gpurun_out/sy
timeout -k 10 400 python -m pytest tests/test_laplace_gpu.py -x -q > gpurun_out/sy/t.log 2>&1; rc=$?; tail -n 3 gpurun_out/sy/t.log; [ $rc -eq 0 ] || exit 1
for v in x6 rows; do
  SNK_SYRK_ORDER=$v timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-extras > gpurun_out/sy/b$v.json 2>gpurun_out/sy/e$v.log || exit 2
  python -c "import json;d=json.load(open('gpurun_out/sy/b$v.json'));print('$v', round(d['d_build_sec'],3), d['d_build']['phase_ms'], round(d['d_build']['roofline']['achieved'],1), d.get('snapshot_gram',{}).get('gram_kernel_ms'))"
done
