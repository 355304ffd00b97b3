#!/bin/bash
# round 5 (r05n): conv_h3f variants A/B: shipping, conv3 LDS-DMA lookahead 6 (la6), persistent
# one-workgroup-per-CU with a group ticket and board prefetch (per), conv3 output stored from the
# accumulators (dir), all three (all): act-forward parity tests on the "all" build, isolated act layers, the headline loop without the D
# build; then the clean MFMA power microbench
set -o pipefail
OUT=gpurun_out/r05n; mkdir -p $OUT
L=$PWD/laplace-dqn-snake-game_amd
SNK_LIB=$L/libsnakehip_all.so timeout -k 10 400 python -u -m pytest tests/test_configs_gpu.py tests/test_configs3_gpu.py "tests/test_qnet_gpu.py::test_dense_h3_act_forward" "tests/test_qnet_gpu.py::test_forward_env_and_act" -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/t_all.log 2>&1; rc=$?
tail -n 3 $OUT/t_all.log; [ $rc -eq 0 ] || exit 2
for v in "" _la6 _per _dir _all; do
  REPS=200 SNK_LIB=$L/libsnakehip$v.so timeout -k 10 240 python -u tools/act_fwd.py > $OUT/act$v.txt 2>&1 || exit 3
  echo "$v $(cat $OUT/act$v.txt)"
done
for v in _all _per _dir _la6 ""; do
  SNK_LIB=$L/libsnakehip$v.so timeout -k 10 300 python bench.py --no-dbuild --no-cpu-baseline --no-configs2 --no-configs3 > $OUT/b$v.json 2> $OUT/b$v.err || exit 4
  python -c "import json;d=json.load(open('$OUT/b$v.json'));print('$v',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'])"
done
timeout -k 10 120 ./tools/mfma_power.bin > $OUT/mfma_power.jsonl 2>&1 || exit 1
echo done
