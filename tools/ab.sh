#!/bin/bash
# Interleaved A/B of library builds or arithmetic knobs on the headline loop (the rounds 4-5
# per-call scripts r04*.sh / r05*.sh folded into one; they are in git history at a51124c).
#   bash tools/ab.sh <tag> <reps> <variant>...
# variant: "lib:<suffix>" runs laplace-dqn-snake-game_amd/libsnakehip<suffix>.so (make variant
# VNAME=<suffix minus _> VDEFS=...; "lib:" is the shipping build), "arith:<knob>=<0|1>" passes
# bench.py --arith. TESTS="<pytest files>" first runs those -m gpu tests on every variant.
# BENCH_ARGS overrides the bench flags (default: the loop without the D build / extras).
set -o pipefail
TAG=${1:?tag}; REPS=${2:-3}; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
L=$PWD/laplace-dqn-snake-game_amd
BA=${BENCH_ARGS:---no-dbuild --no-cpu-baseline --no-configs2 --no-configs3}
env_of() {   # variant -> "SNK_LIB=..." or "" ; args_of: bench args
  case $1 in lib:*) echo "SNK_LIB=$L/libsnakehip${1#lib:}.so";; *) echo "";; esac
}
args_of() { case $1 in arith:*) echo "--arith ${1#arith:}";; *) echo "";; esac; }
if [ -n "$TESTS" ]; then
  for v in "$@"; do
    n=$(echo $v | tr ':=' '__')
    env $(env_of $v) timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 200 --timeout-method thread \
      > $OUT/t_$n.log 2>&1; rc=$?
    echo "$v"; tail -n 2 $OUT/t_$n.log; [ $rc -eq 0 ] || exit 2
  done
fi
for rep in $(seq 0 $((REPS - 1))); do
  for v in "$@"; do
    n=$(echo $v | tr ':=' '__')
    env $(env_of $v) timeout -k 10 300 python bench.py $BA $(args_of $v) > $OUT/b_$n.$rep.json 2> $OUT/b_$n.$rep.err || exit 4
    python -c "import json;d=json.loads(open('$OUT/b_$n.$rep.json').read().strip().splitlines()[-1]);r=d.get('reference_ratio',{});print('$rep $v',d['value'],d['ms_per_step'],(d.get('roofline') or {}).get('avg_launch_ms'),r.get('ms_per_update_marginal'))"
  done
done
echo done
