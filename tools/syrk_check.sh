#!/bin/bash
# h3 Gram: laplace parity tests, D build timing at 16k (h3 vs x6), full-size once: bash tools/syrk_check.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/syrk; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_laplace_gpu.py -q --timeout 120 --timeout-method thread > $OUT/t.log 2>&1; rc=$?; tail -n 3 $OUT/t.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python tools/dbuild.py 16384 2 2>&1 | tail -1 || exit 2
SNK_SYRK=x6 timeout -k 10 120 python tools/dbuild.py 16384 2 2>&1 | tail -1 || exit 3
timeout -k 10 200 python tools/dbuild.py 50000 2 2>&1 | tail -1 || exit 4
