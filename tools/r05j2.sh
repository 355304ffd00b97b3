#!/bin/bash
# round 5 (r05j2): configs[2] L3 with its epilogue bias loaded before the offsets (shipping) vs in
# the epilogue (bl): deep parity on shipping, per-layer forward times (three interleaved rounds)
set -o pipefail
OUT=gpurun_out/r05j2; mkdir -p $OUT
L=$PWD/laplace-dqn-snake-game_amd
timeout -k 10 400 python -u -m pytest tests/test_deep_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/t.log 2>&1; rc=$?
tail -n 2 $OUT/t.log; [ $rc -eq 0 ] || exit 2
for rep in 0 1 2; do
for v in "" _bl; do
  REPS=5 SNK_LIB=$L/libsnakehip$v.so timeout -k 10 240 python -u tools/deep_fwd.py > $OUT/deep$v.$rep.txt 2>&1 || exit 3
  echo "$rep $v $(grep 'deep layers' $OUT/deep$v.$rep.txt)"
done
done
echo done
