#!/bin/bash
# round 5 (r05h): persistent conv_h3f with conv1's weights parked in LDS after the first pass
# (shipping) vs reloaded from L2 every pass (w1g): act tests on shipping, headline A/B
set -o pipefail
OUT=gpurun_out/r05h; mkdir -p $OUT
L=$PWD/laplace-dqn-snake-game_amd
timeout -k 10 400 python -u -m pytest tests/test_configs_gpu.py tests/test_configs3_gpu.py "tests/test_qnet_gpu.py::test_dense_h3_act_forward" "tests/test_qnet_gpu.py::test_env_fused_act_head_bitexact" -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/t.log 2>&1; rc=$?
tail -n 2 $OUT/t.log; [ $rc -eq 0 ] || exit 2
for rep in 0 1 2; do
for v in "" _w1g; do
  SNK_LIB=$L/libsnakehip$v.so timeout -k 10 300 python bench.py --no-dbuild --no-cpu-baseline --no-configs2 --no-configs3 > $OUT/b$v.$rep.json 2> $OUT/b$v.$rep.err || exit 4
  python -c "import json;d=json.load(open('$OUT/b$v.$rep.json'));print('$rep $v',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'])"
done
done
echo done
