#!/bin/bash
# update-path change: GPU suite, unpaired kernel stats, short bench: bash tools/upd_check.sh <tag>
set -o pipefail
TAG=${1:-upd}
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/t.log 2>&1; rc=$?; tail -n 3 $OUT/t.log; [ $rc -eq 0 ] || exit 1
bash tools/unpair2.sh $TAG/up || exit 2
timeout -k 10 300 python bench.py --steps 300 --no-cpu-baseline --no-dbuild > $OUT/b.json 2> $OUT/b.err || exit 3
python -c "import json;d=json.load(open('$OUT/b.json'));print(d['value'], d['ms_per_step'], d['act_forward_ms'])"
