#!/bin/bash
# round 5 (r05be): the update forward's conv3 ring with the offsets split between the two waves
# of a row tile (each wave both column tiles: shipping) against one column tile per wave over
# all offsets (_nks, the ring of r05bb): update + trainer tests on shipping, interleaved runs
set -o pipefail
OUT=gpurun_out/r05be; mkdir -p $OUT
L=$PWD/laplace-dqn-snake-game_amd
timeout -k 10 500 python -u -m pytest tests/test_qnet_gpu.py tests/test_train_parity_gpu.py tests/test_laplace_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/t.log 2>&1; rc=$?
tail -n 2 $OUT/t.log; [ $rc -eq 0 ] || exit 2
for rep in 0 1 2; do
for v in "" _nks; do
  SNK_LIB=$L/libsnakehip$v.so timeout -k 10 300 python bench.py --no-dbuild --no-cpu-baseline --no-configs2 --no-configs3 > $OUT/b$v.$rep.json 2> $OUT/b$v.$rep.err || exit 4
  python -c "import json;d=json.load(open('$OUT/b$v.$rep.json'));r=d['reference_ratio'];print('$rep $v',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],r['ms_per_update_marginal'],r['updates_per_s'])"
done
done
echo done
