set -o pipefail
OUT=gpurun_out/r04a; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_configs3_gpu.py tests/test_deep_gpu.py tests/test_configs_gpu.py -k "configs3 or bound or loss_grad_and_update or stops" -m gpu > $OUT/t.log 2>&1; rc=$?
tail -n 5 $OUT/t.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --no-dbuild --no-configs2 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 3
echo done
