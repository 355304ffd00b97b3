#!/bin/bash
# h3s conv3: targeted tests, full GPU suite, short bench: bash tools/h3_check.sh <tag>
set -o pipefail
TAG=${1:-h3}
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_qnet_gpu.py -v --timeout 120 --timeout-method thread -k "h3s or x6s" -s > $OUT/t1.log 2>&1; rc=$?; tail -n 12 $OUT/t1.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/t.log 2>&1; rc=$?; tail -n 3 $OUT/t.log; [ $rc -eq 0 ] || exit 2
timeout -k 10 300 python bench.py --steps 300 --no-cpu-baseline --no-dbuild > $OUT/b.json 2> $OUT/b.err || exit 3
python -c "import json;d=json.load(open('$OUT/b.json'));print(d['value'], d['ms_per_step'], d['act_forward_ms'], d['roofline'])"
