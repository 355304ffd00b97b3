#!/bin/bash
# round 5 (r05o): conv_h3f A/B, three interleaved rounds of the headline loop (no D build):
# shipping, persistent (per), lookahead 6 (la6), both (perla6); the persistent build's
# act-forward parity first
set -o pipefail
OUT=gpurun_out/r05o; mkdir -p $OUT
L=$PWD/laplace-dqn-snake-game_amd
SNK_LIB=$L/libsnakehip_perla6.so timeout -k 10 400 python -u -m pytest tests/test_configs_gpu.py tests/test_configs3_gpu.py "tests/test_qnet_gpu.py::test_dense_h3_act_forward" "tests/test_qnet_gpu.py::test_forward_env_and_act" -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/t_perla6.log 2>&1; rc=$?
tail -n 2 $OUT/t_perla6.log; [ $rc -eq 0 ] || exit 2
for rep in 0 1 2; do
for v in "" _per _la6 _perla6; do
  SNK_LIB=$L/libsnakehip$v.so timeout -k 10 300 python bench.py --no-dbuild --no-cpu-baseline --no-configs2 --no-configs3  > $OUT/b$v.$rep.json 2> $OUT/b$v.$rep.err || exit 4
  python -c "import json;d=json.load(open('$OUT/b$v.$rep.json'));print('$rep $v',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'])"
done
done
echo done
