#!/bin/bash
# round 5 (r05bl): dense_h3_kernel with 4 waves (64-row blocks, 448 workgroups at 4096, _dw4)
# against 8 waves (128-row blocks, 224 workgroups: shipping): act tests on _dw4, interleaved runs
set -o pipefail
OUT=gpurun_out/r05bl; mkdir -p $OUT
L=$PWD/laplace-dqn-snake-game_amd
SNK_LIB=$L/libsnakehip_dw4.so timeout -k 10 400 python -u -m pytest tests/test_configs_gpu.py tests/test_configs3_gpu.py "tests/test_qnet_gpu.py::test_dense_h3_act_forward" "tests/test_qnet_gpu.py::test_h3f_act_forward_boards_vs_oracle" "tests/test_train_parity_gpu.py::test_bench_graph_trajectory_vs_oracle" -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/t.log 2>&1; rc=$?
tail -n 2 $OUT/t.log; [ $rc -eq 0 ] || exit 2
for rep in 0 1 2; do
for v in "" _dw4; do
  SNK_LIB=$L/libsnakehip$v.so timeout -k 10 300 python bench.py --no-dbuild --no-cpu-baseline --no-configs2 --no-configs3 > $OUT/b$v.$rep.json 2> $OUT/b$v.$rep.err || exit 4
  python -c "import json;d=json.load(open('$OUT/b$v.$rep.json'));print('$rep $v',d['value'],d['ms_per_step'],d['act_forward_ms']['dense1'])"
done
done
echo done
