#!/bin/bash
# round 5 (r05bh): dense_h3_kernel (act Dense1) with the B DMAs issued ahead of every register
# load (no vmcnt(0) drain at position 0) and a3 loaded 2 (shipping), 4 (_ad4) or 6 (_ad6)
# positions ahead, against the tree before (_base): act tests on shipping and _ad6, then
# interleaved headline runs
set -o pipefail
OUT=gpurun_out/r05bh; mkdir -p $OUT
L=$PWD/laplace-dqn-snake-game_amd
for v in "" _ad6; do
SNK_LIB=$L/libsnakehip$v.so timeout -k 10 400 python -u -m pytest tests/test_configs_gpu.py tests/test_configs3_gpu.py "tests/test_qnet_gpu.py::test_dense_h3_act_forward" "tests/test_qnet_gpu.py::test_forward_env_and_act" "tests/test_train_parity_gpu.py::test_bench_graph_trajectory_vs_oracle" -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/t$v.log 2>&1; rc=$?
echo "$v"; tail -n 2 $OUT/t$v.log; [ $rc -eq 0 ] || exit 2
done
for rep in 0 1 2; do
for v in "" _ad4 _ad6 _base; do
  SNK_LIB=$L/libsnakehip$v.so timeout -k 10 300 python bench.py --no-dbuild --no-cpu-baseline --no-configs2 --no-configs3 > $OUT/b$v.$rep.json 2> $OUT/b$v.$rep.err || exit 4
  python -c "import json;d=json.load(open('$OUT/b$v.$rep.json'));a=d['act_forward_ms'];print('$rep $v',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],a['dense1'])"
done
done
echo done
