# round 4: weight-stationary conv3 microbenchmark + PMC evidence (Gram 50k, act forward, configs[2] forward)
set -o pipefail
mkdir -p gpurun_out/r04b
timeout -k 10 60 ./tools/ws_conv3_bench.bin > gpurun_out/r04b/ws.json 2>&1 || exit 1
cat gpurun_out/r04b/ws.json
bash tools/pmc_syrk.sh r04_pmc_syrk 50000 || exit 2
bash tools/pmc_any.sh r04_pmc_h3f tools/act_fwd.py || exit 3
bash tools/pmc_any.sh r04_pmc_deep tools/deep_fwd.py || exit 4
echo done
