#!/bin/bash
# round 5 (r05w): configs[2] L3 on four waves over all 64 channels with the odd-du activation fragments shifted by DPP
# of read from LDS (DL3_SHIFT build, dl3): deep parity tests on that build, per-layer forward
# times of both builds (two interleaved rounds), the configs[2] bench line of both
set -o pipefail
OUT=gpurun_out/r05w; mkdir -p $OUT
L=$PWD/laplace-dqn-snake-game_amd
SNK_LIB=$L/libsnakehip_w4.so timeout -k 10 400 python -u -m pytest tests/test_deep_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/t_w4.log 2>&1; rc=$?
tail -n 2 $OUT/t_w4.log; [ $rc -eq 0 ] || exit 2
for rep in 0 1; do
for v in "" _w4; do
  REPS=5 SNK_LIB=$L/libsnakehip$v.so timeout -k 10 240 python -u tools/deep_fwd.py > $OUT/deep$v.$rep.txt 2>&1 || exit 3
  echo "$rep $v $(grep 'deep layers' $OUT/deep$v.$rep.txt)"
done
done
echo done
