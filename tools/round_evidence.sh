#!/bin/bash
# Round evidence on the GPU box in one call: every -m gpu test, smoke(), the
# default bench line, and a rocprofv3 kernel-trace of the same bench.
# usage: bash tools/round_evidence.sh <tag>   (outputs under gpurun_out/<tag>)
set -o pipefail
TAG=${1:-rx}
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/t.log 2>&1; rc=$?
tail -n 3 $OUT/t.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 2
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 3
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --steps 50 --warmup 10 --repeats 1 --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof.err || exit 4
echo done
