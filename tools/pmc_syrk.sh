#!/bin/bash
# Counter-only passes over a D build (syrk_kernel): bash tools/pmc_syrk.sh <tag> [N]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-pmc_syrk}; N=${2:-16384}; mkdir -p $OUT
timeout -k 10 120 python tools/dbuild.py $N 2 > $OUT/plain.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/p1 -o run -- python tools/dbuild.py $N > $OUT/p1.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $OUT/p2 -o run -- python tools/dbuild.py $N > $OUT/p2.log 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT TCC_MISS TCP_TCC_READ_REQ --output-format csv -d $OUT/p3 -o run -- python tools/dbuild.py $N > $OUT/p3.log 2>&1 || exit 4
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM SQ_WAIT_INST_ANY --output-format csv -d $OUT/p4 -o run -- python tools/dbuild.py $N > $OUT/p4.log 2>&1 || echo p4 failed
echo done
