# round 4: configs[2] L3 ring + pipelined fragments -- deep parity tests, layer times, headline bench (configs2 line)
set -o pipefail
OUT=gpurun_out/r04u; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_deep_gpu.py -m gpu > $OUT/t.log 2>&1; rc=$?
tail -n 2 $OUT/t.log; [ $rc -eq 0 ] || exit 1
REPS=10 timeout -k 10 180 python tools/deep_fwd.py > $OUT/deep.txt 2>&1 || exit 2
cat $OUT/deep.txt | tail -2
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-dbuild --no-cpu-baseline --no-configs3 > $OUT/b.json 2> $OUT/b.err || exit 4
python -c "import json; d=json.load(open('$OUT/b.json')); c=d['configs2']; print(d['value'], c['value'], c['ms_per_step'], c['act_forward_ms'], c['act_forward_tflops'])"
echo done
