#!/bin/bash
# round 5 (r05l): clean MFMA power microbench (f16 vs int8), the update-path GPU tests,
# the headline bench without the D build (update forward with more W1 loads in flight)
set -o pipefail
OUT=gpurun_out/r05l; mkdir -p $OUT
timeout -k 10 120 ./tools/mfma_power.bin > $OUT/mfma_power.jsonl 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_qnet_gpu.py tests/test_train_parity_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/t.log 2>&1; rc=$?
tail -n 2 $OUT/t.log; [ $rc -eq 0 ] || exit 2
timeout -k 10 300 python bench.py --no-dbuild --no-cpu-baseline --no-configs2 --no-configs3 > $OUT/b.json 2> $OUT/b.err || exit 3
echo done
