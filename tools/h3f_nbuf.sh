#!/bin/bash
# conv_h3f_kernel B staging A/B (4 buffers vs SNK_H3F_NBUF=2): parity tests, phase clocks, act timing
set -o pipefail
OUT=gpurun_out/${1:-nbuf}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_qnet_gpu.py -v --timeout 120 --timeout-method thread -k "h3 or x6s or large_batch or act" > $OUT/t1.log 2>&1; rc=$?; tail -n 3 $OUT/t1.log; [ $rc -eq 0 ] || exit 1
for nb in 4 2; do
  SNK_H3F_NBUF=$nb SNK_H3F_DBG=1 timeout -k 10 120 python tools/act_fwd.py > $OUT/dbg$nb.log 2>&1 || exit 2
  grep "h3f dbg" $OUT/dbg$nb.log | head -1
  SNK_H3F_NBUF=$nb REPS=50 timeout -k 10 120 python tools/act_fwd.py > $OUT/act$nb.log 2>&1 || exit 3
  tail -1 $OUT/act$nb.log
done
timeout -k 10 300 python bench.py --no-dbuild --no-cpu-baseline > $OUT/b4.json 2> $OUT/b.err || exit 4
SNK_H3F_NBUF=2 timeout -k 10 300 python bench.py --no-dbuild --no-cpu-baseline > $OUT/b2.json 2>> $OUT/b.err || exit 5
python -c "import json;[print(f, json.load(open('$OUT/'+f))['value'], json.load(open('$OUT/'+f))['act_forward_ms']) for f in ('b4.json','b2.json')]"
