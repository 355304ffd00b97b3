# round 4: full GPU suite + headline bench (no D build) + kernel stats
set -o pipefail
OUT=gpurun_out/r04h; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $OUT/t.log 2>&1; rc=$?
tail -n 2 $OUT/t.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-dbuild --no-configs2 --no-cpu-baseline > $OUT/b.json 2> $OUT/b.err || exit 4
python -c "import json; d=json.load(open('$OUT/b.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['step_kernel'], d['reference_ratio']['updates_per_s'], d['configs3_per_rank']['value'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-dbuild --no-extras --no-configs2 --no-configs3 > $OUT/pb.json 2> $OUT/prof.err || exit 5
python tools/kstats.py $OUT/prof > $OUT/kstats.txt; head -14 $OUT/kstats.txt
echo done
