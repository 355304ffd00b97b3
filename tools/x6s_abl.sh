set -o pipefail
mkdir -p gpurun_out/abl
for m in 0 1 2 4 8 6 14 0; do
  SNK_X6S_DBG=$m timeout -k 10 120 python bench.py --steps 60 --warmup 10 --no-cpu-baseline --no-dbuild > gpurun_out/abl/b$m.json 2>gpurun_out/abl/e$m.log || exit 1
  python -c "import json;d=json.load(open('gpurun_out/abl/b$m.json'));print($m, d['act_forward_ms'])"
done
SNK_X6S=0 timeout -k 10 120 python bench.py --steps 60 --warmup 10 --no-cpu-baseline --no-dbuild > gpurun_out/abl/m16.json 2>/dev/null && python -c "import json;d=json.load(open('gpurun_out/abl/m16.json'));print('m16', d['act_forward_ms'])"
