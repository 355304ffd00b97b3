#!/bin/bash
# h3 conv2: targeted tests, kernel stats, full GPU suite, short bench: bash tools/c2_check.sh <tag>
set -o pipefail
TAG=${1:-c2}
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_qnet_gpu.py -v --timeout 120 --timeout-method thread -k "h3 or x6s or large_batch" -s > $OUT/t1.log 2>&1; rc=$?; tail -n 14 $OUT/t1.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-dbuild > $OUT/pb.json 2> $OUT/prof.err || exit 2
python - "$OUT/prof" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:14]:
    print(f'{float(r["AverageNs"])/1e3:9.1f} us  x{r["Calls"]:>6}  {r["Name"][:90]}')
PY
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/t.log 2>&1; rc=$?; tail -n 3 $OUT/t.log; [ $rc -eq 0 ] || exit 3
timeout -k 10 300 python bench.py --steps 300 --no-cpu-baseline --no-dbuild > $OUT/b.json 2> $OUT/b.err || exit 4
python -c "import json;d=json.load(open('$OUT/b.json'));print(d['value'], d['ms_per_step'], d['act_forward_ms'], d['roofline'])"
