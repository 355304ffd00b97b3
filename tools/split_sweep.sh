#!/bin/bash
mkdir -p gpurun_out/ss
for v in 0 9 0 9; do
  SNK_SPLIT_MIN_KK=$v timeout -k 10 120 python bench.py --steps 400 --no-cpu-baseline --no-dbuild --no-extras > gpurun_out/ss/b$v.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ss/b$v.json'));print($v, round(d['ms_per_step'],4), int(d['value']))"
done
