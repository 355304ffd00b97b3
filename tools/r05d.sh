#!/bin/bash
# round 5 (r05d): Gram lab variants (order / stages per barrier / NB / no-MFMA / no-DMA),
# the -m gpu suite, and the headline bench without the extras (the update's Dense1 now in
# upd_fwd_kernel)
set -o pipefail
OUT=gpurun_out/r05d; mkdir -p $OUT
timeout -k 10 150 ./tools/syrk_lab.bin 50000 2 0x3F3 > $OUT/syrk_lab.jsonl 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/t.log 2>&1; rc=$?
tail -n 3 $OUT/t.log; [ $rc -eq 0 ] || exit 2
timeout -k 10 300 python bench.py --no-dbuild --no-cpu-baseline --no-configs2 > $OUT/b.json 2> $OUT/b.err || exit 3
echo done
