#!/bin/bash
# round 5 (r05t): conv_h3f with its conv3 row tiles balanced over the SIMDs (H3F_BAL, the partial
# last tile split by column tiles): act-forward parity on that build, phase clocks of both, and
# the headline loop (no D build), three interleaved rounds
set -o pipefail
OUT=gpurun_out/r05t; mkdir -p $OUT
L=$PWD/laplace-dqn-snake-game_amd
SNK_LIB=$L/libsnakehip_bal.so timeout -k 10 400 python -u -m pytest tests/test_configs_gpu.py tests/test_configs3_gpu.py "tests/test_qnet_gpu.py::test_dense_h3_act_forward" "tests/test_qnet_gpu.py::test_forward_env_and_act" -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/t_bal.log 2>&1; rc=$?
tail -n 2 $OUT/t_bal.log; [ $rc -eq 0 ] || exit 2
for v in clk clkbal; do
  SNK_LIB=$L/libsnakehip_$v.so timeout -k 10 200 python -u tools/h3f_clocks.py > $OUT/$v.json 2> $OUT/$v.err || exit 1
  echo "$v $(tail -1 $OUT/$v.json)"
done
for rep in 0 1 2; do
for v in "" _bal; do
  SNK_LIB=$L/libsnakehip$v.so timeout -k 10 300 python bench.py --no-dbuild --no-cpu-baseline --no-configs2 --no-configs3 > $OUT/b$v.$rep.json 2> $OUT/b$v.$rep.err || exit 4
  python -c "import json;d=json.load(open('$OUT/b$v.$rep.json'));print('$rep $v',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'])"
done
done
echo done
