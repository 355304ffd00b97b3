#!/bin/bash
# round 5 (r05n): conv_h3f conv3 LDS-DMA lookahead A/B (4 = shipping, 6, 7: make variant),
# isolated act layers and the headline loop without the D build; clean MFMA power microbench
set -o pipefail
OUT=gpurun_out/r05n; mkdir -p $OUT
L=$PWD/laplace-dqn-snake-game_amd
timeout -k 10 120 ./tools/mfma_power.bin > $OUT/mfma_power.jsonl 2>&1 || exit 1
for v in "" _la6 _la7; do
  REPS=200 SNK_LIB=$L/libsnakehip$v.so timeout -k 10 240 python -u tools/act_fwd.py > $OUT/act$v.txt 2>&1 || exit 2
  cat $OUT/act$v.txt
done
for v in _la6 _la7 ""; do
  SNK_LIB=$L/libsnakehip$v.so timeout -k 10 300 python bench.py --no-dbuild --no-cpu-baseline --no-configs2 --no-configs3 > $OUT/b$v.json 2> $OUT/b$v.err || exit 3
  python -c "import json;d=json.load(open('$OUT/b$v.json'));print('$v',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'])"
done
echo done
