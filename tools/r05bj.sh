#!/bin/bash
# round 5 (r05bj): two dependent-load fixes (shipping) against the tree before (_base): the env
# kernel's act head loads epsilon before the Q values (it came after them, behind the early
# returns), and the update forward loads its fused heads' replay fields (slot, then mask / done /
# reward / action) at its start instead of after the arrival ticket: env / update / trajectory
# tests on shipping, interleaved headline runs
set -o pipefail
OUT=gpurun_out/r05bj; mkdir -p $OUT
L=$PWD/laplace-dqn-snake-game_amd
timeout -k 10 400 python -u -m pytest tests/test_env_gpu.py tests/test_configs3_gpu.py tests/test_qnet_gpu.py "tests/test_train_parity_gpu.py" -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/t.log 2>&1; rc=$?
tail -n 2 $OUT/t.log; [ $rc -eq 0 ] || exit 2
for rep in 0 1 2; do
for v in "" _base; do
  SNK_LIB=$L/libsnakehip$v.so timeout -k 10 300 python bench.py --no-dbuild --no-cpu-baseline --no-configs2 --no-configs3 > $OUT/b$v.$rep.json 2> $OUT/b$v.$rep.err || exit 4
  python -c "import json;d=json.load(open('$OUT/b$v.$rep.json'));r=d['reference_ratio'];print('$rep $v',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],r['ms_per_update_marginal'])"
done
done
echo done
