set -e
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/ti_$1.log 2>&1
SNK_LIB=$GRAFT_REPO_ROOT/laplace-dqn-snake-game_amd/libsnakehip_clk.so AMD_SERIALIZE_KERNEL=3 timeout -k 10 300 python -u tools/upd_clocks.py > gpurun_out/updclk_$1.json 2>&1
bash tools/prof_headline.sh $1
