# round 4: conv3_bwd dW dz3 in registers, 3 WG per CU -- gradient parity, clocks, headline bench + kernel stats
set -o pipefail
OUT=gpurun_out/r04p; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_qnet_gpu.py tests/test_train_parity_gpu.py -m gpu > $OUT/t.log 2>&1; rc=$?
tail -n 2 $OUT/t.log; [ $rc -eq 0 ] || exit 1
SNK_LIB=$GRAFT_REPO_ROOT/laplace-dqn-snake-game_amd/libsnakehip_clk.so timeout -k 10 180 python tools/c3b_clocks.py > $OUT/c3b.json 2> $OUT/c3b.err || exit 2
python -c "import json; d=json.load(open('$OUT/c3b.json')); print(d['grid_end_us'], d['max_resident_per_cu'], {k: d['dX'][k]['median'] for k in d['dX']}, {k: d['dW'][k]['median'] for k in d['dW']}); c=d['conv2_bwd']; print('conv2', c['grid_end_us'], {k: c['dX'][k]['median'] for k in c['dX']}, {k: c['dW'][k]['median'] for k in c['dW']})"
SNK_LIB=$GRAFT_REPO_ROOT/laplace-dqn-snake-game_amd/libsnakehip_clk.so timeout -k 10 180 python tools/upd_clocks.py > $OUT/upd.json 2> $OUT/upd.err || exit 3
cat $OUT/upd.json
SNK_LIB=$GRAFT_REPO_ROOT/laplace-dqn-snake-game_amd/libsnakehip_clk.so timeout -k 10 180 python tools/gu_clocks.py > $OUT/gu.json 2> $OUT/gu.err || exit 6
cat $OUT/gu.json
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-dbuild --no-configs2 --no-cpu-baseline > $OUT/b.json 2> $OUT/b.err || exit 4
python -c "import json; d=json.load(open('$OUT/b.json')); print(d['value'], d['ms_per_step'], d['reference_ratio']['updates_per_s'], d['reference_ratio']['ms_per_update_marginal'], d['configs3_per_rank']['value'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-dbuild --no-extras --no-configs2 --no-configs3 > $OUT/pb.json 2> $OUT/prof.err || exit 5
python tools/kstats.py $OUT/prof > $OUT/kstats.txt; head -14 $OUT/kstats.txt
echo done
