#!/bin/bash
# Counters of the act-forward kernels: counter-only passes (no trace domains)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${PMC_TAG:-pmc_act2}; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --pmc TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TCP_PENDING_STALL_CYCLES TCP_TCC_READ_REQ TCP_READ_TAGCONFLICT_STALL_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $OUT/p3 -o run -- python tools/act_fwd.py > $OUT/p3.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc TCC_HIT TCC_MISS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $OUT/p4 -o run -- python tools/act_fwd.py > $OUT/p4.log 2>&1 || exit 2
echo done
