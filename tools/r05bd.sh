#!/bin/bash
# round 5 (r05bd): phase clocks of the B = 64 update chain after the 3-offset conv3 ring
# (clocks build): update forward, conv3 backward, grad_update
set -o pipefail
OUT=gpurun_out/r05bd; mkdir -p $OUT
export SNK_LIB=$PWD/laplace-dqn-snake-game_amd/libsnakehip_clk.so
timeout -k 10 200 python tools/upd_clocks.py > $OUT/upd_clocks.json 2> $OUT/upd.err || exit 1
timeout -k 10 200 python tools/c3b_clocks.py > $OUT/c3b_clocks.json 2> $OUT/c3b.err || exit 2
timeout -k 10 200 python tools/gu_clocks.py > $OUT/gu_clocks.json 2> $OUT/gu.err || exit 3
cat $OUT/upd_clocks.json; echo; cat $OUT/c3b_clocks.json | head -c 1500; echo; cat $OUT/gu_clocks.json | head -c 1500
