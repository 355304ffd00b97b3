# round 4: conv_h3f a3max via DPP rows -- forward/trainer parity, headline bench + kernel stats
set -o pipefail
OUT=gpurun_out/r04za; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_qnet_gpu.py tests/test_train_parity_gpu.py -m gpu > $OUT/t.log 2>&1; rc=$?
tail -n 2 $OUT/t.log; [ $rc -eq 0 ] || exit 1
SNK_LIB=$GRAFT_REPO_ROOT/laplace-dqn-snake-game_amd/libsnakehip_clk.so timeout -k 10 180 python tools/h3f_clocks.py > $OUT/h3f.json 2> $OUT/h3f.err || exit 3
cat $OUT/h3f.json
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-dbuild --no-configs2 --no-cpu-baseline > $OUT/b.json 2> $OUT/b.err || exit 4
python -c "import json; d=json.load(open('$OUT/b.json')); print(d['value'], d['ms_per_step'], d['act_forward_ms'], d['reference_ratio']['updates_per_s'], d['configs3_per_rank']['value'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-dbuild --no-extras --no-configs2 --no-configs3 > $OUT/pb.json 2> $OUT/prof.err || exit 5
python tools/kstats.py $OUT/prof > $OUT/kstats.txt; head -16 $OUT/kstats.txt
echo done
