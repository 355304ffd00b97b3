# round 4: lap_act rings + conv_h3f LDS-DMA B staging: parity, lap sampling timing, headline + rocprof stats
set -o pipefail
OUT=gpurun_out/r04d; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_laplace_gpu.py tests/test_qnet_gpu.py tests/test_configs3_gpu.py tests/test_configs_gpu.py tests/test_train_parity_gpu.py tests/test_env_gpu.py tests/test_deep_gpu.py -m gpu > $OUT/t.log 2>&1; rc=$?
tail -n 3 $OUT/t.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python tools/lap_sampling.py > $OUT/ls.json 2>&1 || exit 2
tail -2 $OUT/ls.json
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-dbuild --no-configs2 --no-cpu-baseline > $OUT/b.json 2> $OUT/b.err || exit 3
python -c "import json; d=json.load(open('$OUT/b.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d.get('reference_ratio'), d['configs3_per_rank']['value'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-dbuild --no-extras --no-configs2 --no-configs3 > $OUT/pb.json 2> $OUT/prof.err || exit 4
python tools/kstats.py $OUT/prof | head -16
echo done
