#!/bin/bash
# configs[2] iteration: the deep-net GPU tests, the bench line with the configs[2]
# extra (no D build, no CPU baseline), and its kernel-trace stats.
# usage: bash tools/gpu_deep.sh <tag>   (outputs under gpurun_out/<tag>)
set -o pipefail
TAG=${1:-deep}
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_deep_gpu.py -m gpu -v -s --timeout 120 --timeout-method thread > $OUT/t.log 2>&1; rc=$?
tail -n 3 $OUT/t.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --repeats 3 --no-extras --no-dbuild --no-cpu-baseline > $OUT/b.json 2> $OUT/b.err || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --steps 10 --warmup 3 --repeats 1 --no-extras --no-dbuild --no-cpu-baseline > $OUT/pb.json 2> $OUT/prof.err || exit 3
echo done
