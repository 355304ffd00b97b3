#!/bin/bash
# round 5 (r05y): the trainer's grad_update writes the next act forward's split weight images
# (split_chain; w3_split_kernel once per captured graph, exponents with 4 bits of headroom):
# the qnet / configs / trainer tests, then the headline loop (no D build) split_chain=1 / 0,
# three interleaved rounds
set -o pipefail
OUT=gpurun_out/r05y; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_qnet_gpu.py tests/test_configs_gpu.py tests/test_configs3_gpu.py tests/test_train_parity_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/t.log 2>&1; rc=$?
tail -n 2 $OUT/t.log; [ $rc -eq 0 ] || exit 2
for rep in 0 1 2; do
for v in 1 0; do
  timeout -k 10 300 python bench.py --no-dbuild --no-cpu-baseline --no-configs2 --no-configs3 --arith split_chain=$v > $OUT/b$v.$rep.json 2> $OUT/b$v.$rep.err || exit 4
  python -c "import json;d=json.load(open('$OUT/b$v.$rep.json'));print('$rep split_chain=$v',d['value'],d['ms_per_step'],d.get('reference_ratio',{}).get('ms_per_update_marginal'))"
done
done
echo done
