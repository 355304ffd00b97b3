#!/bin/bash
# Counter-only rocprofv3 passes (one counter group per run, no tracing) over the kernels the
# bench line prices, as shipped: the headline training loop (tools/train_iter.py: conv_h3f,
# dense_h3, env_step and the five B = 64 update kernels) and the configs[2] act forward
# (tools/deep_fwd.py). bash tools/pmc_round.sh <tag>  ->  gpurun_out/<tag>_{loop,deep}/p1..p4
# Summaries: python tools/pmc_summary.py gpurun_out/<tag>_loop <out.json> [kernels...];
# traffic: python tools/traffic.py gpurun_out/<tag>_loop <kernel> <out.json> [alg bytes]
# (the D(50k) Gram: tools/pmc_syrk.sh <tag> 50000 and tools/pmc_traffic.sh <tag> syrk)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
TAG=${1:-pmc}
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
P2="FETCH_SIZE GRBM_GUI_ACTIVE"
P3="WRITE_SIZE TCC_HIT TCC_MISS"
P4="SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_SALU SQ_WAVES"
for tgt in loop:tools/train_iter.py deep:tools/deep_fwd.py; do
  name=${tgt%%:*}; script=${tgt#*:}; OUT=gpurun_out/${TAG}_$name; mkdir -p $OUT
  i=1
  for grp in "$P1" "$P2" "$P3" "$P4"; do
    timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python $script > $OUT/p$i.log 2>&1 || exit $i
    i=$((i + 1))
  done
done
echo done
