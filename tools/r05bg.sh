#!/bin/bash
# round 5 (r05bg): the update forward's Dense1 (phase 4) skips the W1 rows whose a3 value is 0
# (range-checked buffer loads, shipping) against loading every row (_noskip): update + trainer
# tests on shipping, interleaved headline runs, phase clocks of the clocks build
set -o pipefail
OUT=gpurun_out/r05bg; mkdir -p $OUT
L=$PWD/laplace-dqn-snake-game_amd
timeout -k 10 500 python -u -m pytest tests/test_qnet_gpu.py tests/test_train_parity_gpu.py tests/test_laplace_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/t.log 2>&1; rc=$?
tail -n 2 $OUT/t.log; [ $rc -eq 0 ] || exit 2
SNK_LIB=$L/libsnakehip_clk.so timeout -k 10 200 python tools/upd_clocks.py > $OUT/upd_clocks.json 2> $OUT/upd.err || exit 3
python -c "
import json;t=open('$OUT/upd_clocks.json').read();d=json.loads(t[t.index('{'):])
print('clk', {k:round(v['median'],2) for k,v in d.items() if isinstance(v,dict) and 'median' in v})"
for rep in 0 1 2; do
for v in "" _noskip; do
  SNK_LIB=$L/libsnakehip$v.so timeout -k 10 300 python bench.py --no-dbuild --no-cpu-baseline --no-configs2 --no-configs3 > $OUT/b$v.$rep.json 2> $OUT/b$v.$rep.err || exit 4
  python -c "import json;d=json.load(open('$OUT/b$v.$rep.json'));r=d['reference_ratio'];print('$rep $v',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],r['ms_per_update_marginal'],r['updates_per_s'])"
done
done
echo done
