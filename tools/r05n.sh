#!/bin/bash
# round 5 (r05n): the update forward's phase-5 hand-off by sc1 stores / loads (shipping) against
# the acq_rel ticket (acq); conv_h3f variants: conv3 LDS-DMA lookahead 6 (la6), persistent
# one-workgroup-per-CU with a group ticket and board prefetch (per), conv3 output stored from the
# accumulators (dir), all three (all). Parity: the update-path tests on the shipping build, the
# act-forward tests on "all"; then isolated act layers and the headline loop (no D build) per
# build; the clean MFMA power microbench last
set -o pipefail
OUT=gpurun_out/r05n; mkdir -p $OUT
L=$PWD/laplace-dqn-snake-game_amd
timeout -k 10 500 python -u -m pytest tests/test_qnet_gpu.py tests/test_train_parity_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/t_ship.log 2>&1; rc=$?
tail -n 2 $OUT/t_ship.log; [ $rc -eq 0 ] || exit 2
SNK_LIB=$L/libsnakehip_all.so timeout -k 10 400 python -u -m pytest tests/test_configs_gpu.py tests/test_configs3_gpu.py "tests/test_qnet_gpu.py::test_dense_h3_act_forward" "tests/test_qnet_gpu.py::test_forward_env_and_act" -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/t_all.log 2>&1; rc=$?
tail -n 2 $OUT/t_all.log; [ $rc -eq 0 ] || exit 2
for v in "" _la6 _per _dir _all; do
  REPS=200 SNK_LIB=$L/libsnakehip$v.so timeout -k 10 240 python -u tools/act_fwd.py > $OUT/act$v.txt 2>&1 || exit 3
  echo "$v $(cat $OUT/act$v.txt)"
done
for v in _all "" _acq _per _dir _la6; do
  SNK_LIB=$L/libsnakehip$v.so timeout -k 10 300 python bench.py --no-dbuild --no-cpu-baseline --no-configs2 --no-configs3 > $OUT/b$v.json 2> $OUT/b$v.err || exit 4
  python -c "import json;d=json.load(open('$OUT/b$v.json'));print('$v',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],d.get('reference_ratio',{}).get('ms_per_update_marginal'))"
done
timeout -k 10 120 ./tools/mfma_power.bin > $OUT/mfma_power.jsonl 2>&1 || exit 1
echo done
