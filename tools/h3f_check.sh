#!/bin/bash
# fused conv2+conv3: targeted tests, phase clocks, full GPU suite, short bench: bash tools/h3f_check.sh <tag>
set -o pipefail
TAG=${1:-h3f}
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_qnet_gpu.py -v --timeout 120 --timeout-method thread -k "h3 or x6s or large_batch" -s > $OUT/t1.log 2>&1; rc=$?; tail -n 14 $OUT/t1.log; [ $rc -eq 0 ] || exit 1
SNK_H3F_DBG=1 timeout -k 10 120 python tools/act_fwd.py > $OUT/dbg.log 2>&1 || exit 2
grep "h3f dbg" $OUT/dbg.log | head -3
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/t.log 2>&1; rc=$?; tail -n 3 $OUT/t.log; [ $rc -eq 0 ] || exit 3
timeout -k 10 300 python bench.py --steps 300 --no-cpu-baseline --no-dbuild > $OUT/b.json 2> $OUT/b.err || exit 4
python -c "import json;d=json.load(open('$OUT/b.json'));print(d['value'], d['ms_per_step'], d['act_forward_ms'], d['roofline'])"
