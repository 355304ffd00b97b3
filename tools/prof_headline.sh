#!/bin/bash
# headline bench (no extras) + rocprofv3 kernel-trace stats of the same: bash tools/prof_headline.sh <tag>
set -o pipefail
TAG=${1:-h}
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-extras --no-dbuild --no-configs2 --no-cpu-baseline > $OUT/b.json 2> $OUT/b.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-dbuild --no-extras --no-configs2 > $OUT/pb.json 2> $OUT/prof.err || exit 2
echo done
