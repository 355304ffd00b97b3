#!/bin/bash
# tests + bench + kernel-trace stats (no counters): bash tools/quick_prof.sh <tag>
set -o pipefail
TAG=${1:-q}
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $OUT/t.log 2>&1; echo "tests rc=$?"; tail -n 3 $OUT/t.log
timeout -k 10 300 python bench.py --steps 300 --no-cpu-baseline --no-dbuild > $OUT/b.json 2> $OUT/b.err || exit 1
python -c "import json;d=json.load(open('$OUT/b.json'));print(d['value'], d['ms_per_step'], d['act_forward_ms'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-dbuild --no-extras > $OUT/pb.json 2> $OUT/prof.err || exit 2
echo done
