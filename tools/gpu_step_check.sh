# GPU: full parity suite, step roofline rows, step phase clocks
set -e
export PYTHONUNBUFFERED=1
TAG=${1:-x}
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/ts_$TAG.log 2>&1
timeout -k 10 300 python -u tools/step_roofline.py > gpurun_out/step_$TAG.jsonl 2>&1
for cfg in "262144 20 0" "65536 20 0" "4096 12 1"; do
  SNK_LIB=$GRAFT_REPO_ROOT/laplace-dqn-snake-game_amd/libsnakehip_clk.so timeout -k 10 120 python -u tools/step_clocks.py $cfg >> gpurun_out/clks_$TAG.jsonl 2>&1
done
