#!/bin/bash
# round 5 (r05s): conv_h3f phase clocks (measurement builds, tools/h3f_clocks.py): the shipping
# kernel and its conv3 offset loop without LDS-DMA (v1), barriers (v2), MFMAs (v3), fragment reads (v4)
set -o pipefail
OUT=gpurun_out/r05s; mkdir -p $OUT
L=$PWD/laplace-dqn-snake-game_amd
for v in clk clkv1 clkv2 clkv3 clkv4 clk; do
  SNK_LIB=$L/libsnakehip_$v.so timeout -k 10 200 python -u tools/h3f_clocks.py > $OUT/$v.json 2> $OUT/$v.err || exit 1
  echo "$v $(tail -1 $OUT/$v.json)"
done
echo done
