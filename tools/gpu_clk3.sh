set -e
export PYTHONUNBUFFERED=1
export SNK_LIB=$GRAFT_REPO_ROOT/laplace-dqn-snake-game_amd/libsnakehip_clk.so
AMD_SERIALIZE_KERNEL=3 HIP_LAUNCH_BLOCKING=1 timeout -k 10 300 python -u tools/upd_clocks.py > gpurun_out/updclk_$1.json 2>&1
