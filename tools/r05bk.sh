#!/bin/bash
# round 5 (r05bk): conv_h3f's conv1 on the matrix cores (h3 split, _c1mfma) against the VALU form
# (shipping): act tests on shipping, interleaved
# headline runs
set -o pipefail
OUT=gpurun_out/r05bk; mkdir -p $OUT
L=$PWD/laplace-dqn-snake-game_amd
timeout -k 10 400 python -u -m pytest tests/test_configs_gpu.py tests/test_configs3_gpu.py "tests/test_qnet_gpu.py::test_dense_h3_act_forward" "tests/test_qnet_gpu.py::test_h3f_act_forward_boards_vs_oracle" "tests/test_qnet_gpu.py::test_forward_env_and_act" "tests/test_qnet_gpu.py::test_forward_random_vs_oracle" "tests/test_qnet_gpu.py::test_env_fused_act_head_bitexact" "tests/test_train_parity_gpu.py::test_bench_graph_trajectory_vs_oracle" -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/t.log 2>&1; rc=$?
tail -n 2 $OUT/t.log; [ $rc -eq 0 ] || exit 2
SNK_LIB=$L/libsnakehip_c1mfma.so timeout -k 10 300 python -u -m pytest tests/test_configs_gpu.py tests/test_configs3_gpu.py "tests/test_qnet_gpu.py::test_h3f_act_forward_boards_vs_oracle" "tests/test_qnet_gpu.py::test_forward_env_and_act" "tests/test_qnet_gpu.py::test_env_fused_act_head_bitexact" "tests/test_train_parity_gpu.py::test_bench_graph_trajectory_vs_oracle" -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/t_c1mfma.log 2>&1; rc=$?
tail -n 1 $OUT/t_c1mfma.log; [ $rc -eq 0 ] || exit 3
for rep in 0 1 2; do
for v in "" _c1mfma; do
  SNK_LIB=$L/libsnakehip$v.so timeout -k 10 300 python bench.py --no-dbuild --no-cpu-baseline --no-configs2 --no-configs3 > $OUT/b$v.$rep.json 2> $OUT/b$v.$rep.err || exit 4
  python -c "import json;d=json.load(open('$OUT/b$v.$rep.json'));print('$rep $v',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'])"
done
done
echo done
