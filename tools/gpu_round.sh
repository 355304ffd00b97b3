# one GPU call: full -m gpu suite, smoke, step phase clocks, headline bench (no extras)
set -e
export PYTHONUNBUFFERED=1
TAG=${1:-x}
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/t_$TAG.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
for cfg in "262144 20 0" "65536 20 0" "4096 12 1"; do
  SNK_LIB=$GRAFT_REPO_ROOT/laplace-dqn-snake-game_amd/libsnakehip_clk.so timeout -k 10 120 python -u tools/step_clocks.py $cfg >> gpurun_out/clk_$TAG.jsonl 2>&1
done
timeout -k 10 600 python -u bench.py --steps 50 --warmup 10 --no-extras --no-dbuild --no-configs2 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
