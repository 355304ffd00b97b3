#!/bin/bash
# Counter-only passes over the step kernel at 262,144 x 20x20: bash tools/pmc_step.sh <tag> <store 0|1>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-pmc_step}; mkdir -p $OUT
ST=${2:-0}
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/p0 -o run -- python tools/step_only.py 262144 20 $ST > $OUT/p0.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $OUT/p2 -o run -- python tools/step_only.py 262144 20 $ST > $OUT/p2.log 2>&1 || exit 2
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE TCC_HIT TCC_MISS --output-format csv -d $OUT/p3 -o run -- python tools/step_only.py 262144 20 $ST > $OUT/p3.log 2>&1 || exit 3
echo done
