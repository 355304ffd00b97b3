#!/bin/bash
# bench ms/step for a few backward-GEMM planner settings
mkdir -p gpurun_out/gs
for cfg in "4096 32" "8192 16" "16384 16" "8192 8"; do
  set -- $cfg
  SNK_GEMM_WAVES=$1 SNK_GEMM_MINK=$2 timeout -k 10 120 python bench.py --steps 300 --no-cpu-baseline --no-dbuild --no-extras > gpurun_out/gs/b_$1_$2.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/gs/b_$1_$2.json'));print('$1 $2', round(d['ms_per_step'],4), int(d['value']))"
done
