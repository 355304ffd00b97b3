#!/bin/bash
# Counter-only passes (as pmc_h3.sh) over any profiling target:
#   bash tools/pmc_any.sh <tag> <python script> [args...]
# then: python tools/pmc_summary.py gpurun_out/<tag> <out.json> [kernel substrings]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-pmc_any}; shift; mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/p1 -o run -- python "$@" > $OUT/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $OUT/p2 -o run -- python "$@" > $OUT/p2.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_SALU SQ_WAVES --output-format csv -d $OUT/p4 -o run -- python "$@" > $OUT/p4.log 2>&1 || echo "p4 failed"
echo done
