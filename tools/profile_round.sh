#!/bin/bash
# Round profile: full bench line + rocprofv3 kernel-trace stats of the same command.
# usage (on the GPU box): bash tools/profile_round.sh <tag>
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --steps 50 --warmup 10 --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof.err || exit 2
echo done
