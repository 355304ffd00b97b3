#!/bin/bash
# conv3_bwd_kernel phase clocks (eager, once): bash tools/c3_dbg.sh
set -o pipefail
mkdir -p gpurun_out/c3dbg
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
SNK_C3_DBG=1 timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-dbuild --no-extras --no-graph > gpurun_out/c3dbg/b.json 2> gpurun_out/c3dbg/err.log; rc=$?
grep "c3bwd dbg" gpurun_out/c3dbg/err.log; exit $rc
