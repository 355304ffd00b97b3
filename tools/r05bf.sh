#!/bin/bash
# round 5 (r05bf): what bounds the update forward's conv3 and Dense1 phases: phase clocks of the
# clocks build against measurement builds (wrong results by design) without the conv3 ring's
# refill DMAs (_clkm1) and without Dense1's W1 loads (_clkm2)
set -o pipefail
OUT=gpurun_out/r05bf; mkdir -p $OUT
L=$PWD/laplace-dqn-snake-game_amd
for rep in 0 1; do
for v in _clk _clkm1 _clkm2; do
SNK_LIB=$L/libsnakehip$v.so timeout -k 10 200 python tools/upd_clocks.py > $OUT/upd$v.$rep.json 2> $OUT/upd$v.$rep.err || exit 1
python -c "
import json;t=open('$OUT/upd$v.$rep.json').read();d=json.loads(t[t.index('{'):])
print('$rep $v', {k:round(v['median'],2) for k,v in d.items() if isinstance(v,dict) and 'median' in v})"
done
done
