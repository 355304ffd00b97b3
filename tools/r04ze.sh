# round 4: dense_h3 with a3 three positions ahead -- forward / trainer / configs parity, bench, kernel stats
set -o pipefail
OUT=gpurun_out/r04ze; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_qnet_gpu.py tests/test_configs_gpu.py tests/test_train_parity_gpu.py -m gpu > $OUT/t.log 2>&1; rc=$?
tail -n 2 $OUT/t.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-dbuild --no-configs2 --no-cpu-baseline --no-configs3 > $OUT/b20.json 2> $OUT/b20.err || exit 5
python -c "import json; d=json.load(open('$OUT/b20.json')); print('steps20', d['value'], d['ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-dbuild --no-extras --no-configs2 --no-configs3 > $OUT/pb.json 2> $OUT/prof.err || exit 6
python tools/kstats.py $OUT/prof > $OUT/kstats.txt; head -6 $OUT/kstats.txt
echo done
