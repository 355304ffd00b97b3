set -o pipefail
mkdir -p gpurun_out/c1
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/c1/t.log 2>&1; rc=$?; tail -n 3 gpurun_out/c1/t.log; [ $rc -eq 0 ] || exit 1
for v in 256 512 1024 256; do
  SNK_C1_DIV=$v timeout -k 10 120 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-dbuild > gpurun_out/c1/b$v.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/c1/b$v.json'));a=d['act_forward_ms'];print($v, round(d['ms_per_step'],4), int(d['value']), round(a['conv1']*1e3,1), round(a['conv2']*1e3,1), round(a['conv3']*1e3,1))"
done
