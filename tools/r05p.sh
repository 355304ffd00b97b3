#!/bin/bash
# round 5 (r05p): the act head fused into dense_h3_kernel's tail: its bit-exactness test and the
# act / update-path tests, then the headline loop (no D build) fused vs head_kernel, two
# interleaved rounds, and the rocprof kernel stats of the fused loop
set -o pipefail
OUT=gpurun_out/r05p; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_qnet_gpu.py tests/test_configs_gpu.py tests/test_configs3_gpu.py tests/test_train_parity_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/t.log 2>&1; rc=$?
tail -n 2 $OUT/t.log; [ $rc -eq 0 ] || exit 2
for rep in 0 1; do
for v in 1 0; do
  timeout -k 10 300 python bench.py --no-dbuild --no-cpu-baseline --no-configs2 --no-configs3 --arith act_head=$v > $OUT/b$v.$rep.json 2> $OUT/b$v.$rep.err || exit 4
  python -c "import json;d=json.load(open('$OUT/b$v.$rep.json'));print('$rep act_head=$v',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],d.get('reference_ratio',{}).get('ms_per_update_marginal'))"
done
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python bench.py --no-dbuild --no-cpu-baseline --no-configs2 --no-configs3 --no-extras --steps 20 --repeats 2 > $OUT/prof.log 2>&1 || exit 5
echo done
