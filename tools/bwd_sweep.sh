set -o pipefail
mkdir -p gpurun_out/bw
run() {  # tag, env...
  tag=$1; shift
  env "$@" timeout -k 10 120 python bench.py --steps 150 --warmup 10 --no-cpu-baseline --no-dbuild --no-extras > gpurun_out/bw/$tag.json 2>gpurun_out/bw/$tag.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/bw/$tag.json'));print('$tag', round(d['ms_per_step'],4), int(d['value']))"
}
run base SNK_X=0
run dx16 SNK_DX_SPLITS=16
run dx36 SNK_DX_SPLITS=36
run kw8k SNK_KW_WAVES=8192
run kw16k SNK_KW_WAVES=16384
run kw16k8 SNK_KW_WAVES=16384 SNK_KW_MINK=8
run dx16kw16k SNK_DX_SPLITS=16 SNK_KW_WAVES=16384
run gw16k SNK_GEMM_WAVES=16384
run base2 SNK_X=0
