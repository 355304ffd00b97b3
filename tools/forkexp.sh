mkdir -p gpurun_out/fx
for m in 0 1 2 4 8 16 31 3; do
  SNK_FORK=$m timeout -k 10 120 python bench.py --steps 300 --no-cpu-baseline --no-dbuild --no-extras > gpurun_out/fx/b$m.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/fx/b$m.json'));print($m, round(d['ms_per_step'],4), int(d['value']))"
done
