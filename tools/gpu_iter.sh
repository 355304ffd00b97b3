# GPU: full parity suite + headline bench + rocprof kernel stats: bash tools/gpu_iter.sh <tag>
set -e
export PYTHONUNBUFFERED=1
TAG=${1:-x}
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/ti_$TAG.log 2>&1
bash tools/prof_headline.sh $TAG
