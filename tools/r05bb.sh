#!/bin/bash
# round 5 (r05bb): the update forward's conv2 fragments read one pair ahead (shipping) or next to
# their MFMAs (_c2old), and its conv3 ring with 2 or 3 offsets per barrier step (UPDF_KS; shipping
# 1): update tests on shipping and both ring variants, then interleaved headline runs
set -o pipefail
OUT=gpurun_out/r05bb; mkdir -p $OUT
L=$PWD/laplace-dqn-snake-game_amd
for v in "" _ks2 _ks3; do
SNK_LIB=$L/libsnakehip$v.so timeout -k 10 400 python -u -m pytest tests/test_qnet_gpu.py tests/test_train_parity_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/t$v.log 2>&1; rc=$?
echo "$v"; tail -n 2 $OUT/t$v.log; [ $rc -eq 0 ] || exit 2
done
for rep in 0 1 2; do
for v in "" _c2old _ks2 _ks3; do
  SNK_LIB=$L/libsnakehip$v.so timeout -k 10 300 python bench.py --no-dbuild --no-cpu-baseline --no-configs2 --no-configs3 > $OUT/b$v.$rep.json 2> $OUT/b$v.$rep.err || exit 4
  python -c "import json;d=json.load(open('$OUT/b$v.$rep.json'));r=d['reference_ratio'];print('$rep $v',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],r['ms_per_update_marginal'],r['updates_per_s'])"
done
done
echo done
