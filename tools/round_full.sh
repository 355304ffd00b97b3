#!/bin/bash
# Round evidence in one call: GPU tests, smoke, default bench, kernel-trace profile of
# the same bench, FETCH/WRITE passes over the act forward. bash tools/round_full.sh <tag>
set -o pipefail
TAG=${1:-rf}
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/t.log 2>&1; rc=$?; tail -n 4 $OUT/t.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 2
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 3
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['act_forward_ms'], d['d_build_sec'], d['cpu_baseline']['value'])"
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --steps 50 --warmup 10 --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof.err || exit 4
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc/p2 -o run -- python tools/act_fwd.py > $OUT/p2.log 2>&1 || exit 5
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE TCC_HIT TCC_MISS --output-format csv -d $OUT/pmc/p3 -o run -- python tools/act_fwd.py > $OUT/p3.log 2>&1 || exit 6
SNK_GRAPH_UNROLL=1 timeout -k 10 300 python bench.py --no-dbuild --no-cpu-baseline --no-extras > $OUT/bench_u1.json 2>> $OUT/bench.err || exit 7
echo done
