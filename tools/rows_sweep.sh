#!/bin/bash
mkdir -p gpurun_out/rs
timeout -k 10 300 python -m pytest tests/test_qnet_gpu.py -x -q > gpurun_out/rs/t.log 2>&1; echo "tests rc=$?"; tail -n 1 gpurun_out/rs/t.log
for rows in 128 256 128 256; do
  SNK_M16_ROWS=$rows timeout -k 10 120 python bench.py --steps 300 --no-cpu-baseline --no-dbuild > gpurun_out/rs/b$rows.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/rs/b$rows.json'));print($rows, round(d['ms_per_step'],4), int(d['value']), round(d['act_forward_ms']['conv3']*1e3,1))"
done
