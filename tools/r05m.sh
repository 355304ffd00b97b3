#!/bin/bash
# round 5 (r05m): the Gram's cost split on DENSE rows (the D(50k) Jacobian's kind): library
# kernel, no-MFMA, no-DMA, half-DMA, 256x128 fp32-only
set -o pipefail
OUT=gpurun_out/r05m; mkdir -p $OUT
timeout -k 10 200 ./tools/syrk_lab.bin 50000 2 0x481031 0 > $OUT/syrk_lab.jsonl 2>&1 || exit 1
echo done
