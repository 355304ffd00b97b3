#!/bin/bash
# tests + bench + kernel-trace profile + counter passes: bash tools/h3_round.sh <tag>
set -o pipefail
TAG=${1:-rr}
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/t.log 2>&1; rc=$?; tail -n 3 $OUT/t.log; [ $rc -eq 0 ] || exit 1
bash tools/pmc_h3.sh $TAG/pmc || exit 2
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 3
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['d_build_sec'], d['cpu_baseline']['value'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --steps 50 --warmup 10 --no-cpu-baseline > $OUT/pb.json 2> $OUT/prof.err || exit 4
echo done
