set -e
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu -k "env or stats or trajectory or configs1 or laplace_sampling or smoke" > gpurun_out/t3.log 2>&1
timeout -k 10 300 python -u tools/step_roofline.py > gpurun_out/step3.jsonl 2>&1
bash tools/pmc_step.sh pmc_step_pure3 0
