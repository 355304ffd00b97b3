# round 4: conv3_bwd phase clocks + after-fix PMC passes (act forward, configs[2] forward)
set -o pipefail
OUT=gpurun_out/r04j; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
SNK_LIB=$GRAFT_REPO_ROOT/laplace-dqn-snake-game_amd/libsnakehip_clk.so timeout -k 10 180 python tools/c3b_clocks.py > $OUT/c3b.json 2> $OUT/c3b.err || exit 1
cat $OUT/c3b.json
bash tools/pmc_traffic.sh r04j h3f || exit 2
bash tools/pmc_traffic.sh r04j deep || exit 3
bash tools/pmc_any.sh r04j_h3fpmc tools/act_fwd.py || exit 4
bash tools/pmc_any.sh r04j_deeppmc tools/deep_fwd.py || exit 5
echo done
