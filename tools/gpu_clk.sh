set -e
export SNK_LIB=$GRAFT_REPO_ROOT/laplace-dqn-snake-game_amd/libsnakehip_clk.so
for cfg in "262144 20 0" "65536 20 0" "262144 20 1" "4096 12 1"; do
  timeout -k 10 120 python -u tools/step_clocks.py $cfg >> gpurun_out/clk1.jsonl 2>&1
done
