#!/bin/bash
# HBM traffic of the two MFMA kernels the bench line prices, from separate counter-only
# rocprofv3 passes (FETCH_SIZE | WRITE_SIZE): bash tools/pmc_traffic.sh <tag>
#   act forward at 4096 x 12x12 (conv_h3f_kernel)      -> gpurun_out/<tag>_h3f/p2, p3
#   Jacobian-Gram D build at n = 50,000 (syrk_h3q_kernel) -> gpurun_out/<tag>_syrk/p2, p3
#   configs[2] act forward at 65,536 x 20x20 (deep_conv3_kernel, deep_front_kernel) -> gpurun_out/<tag>_deep/p2, p3
#   (a second argument restricts the run to one of h3f | syrk | deep)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
TAG=${1:-pmc}
ONLY=${2:-all}
A=gpurun_out/${TAG}_h3f; S=gpurun_out/${TAG}_syrk; P=gpurun_out/${TAG}_deep; mkdir -p $A $S $P
if [ $ONLY = all ] || [ $ONLY = h3f ]; then
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $A/p2 -o run -- python tools/act_fwd.py > $A/p2.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE TCC_HIT TCC_MISS --output-format csv -d $A/p3 -o run -- python tools/act_fwd.py > $A/p3.log 2>&1 || exit 2
fi
if [ $ONLY = all ] || [ $ONLY = syrk ]; then
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $S/p2 -o run -- python tools/dbuild.py 50000 > $S/p2.log 2>&1 || exit 3
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE TCC_HIT TCC_MISS --output-format csv -d $S/p3 -o run -- python tools/dbuild.py 50000 > $S/p3.log 2>&1 || exit 4
fi
if [ $ONLY = all ] || [ $ONLY = deep ]; then
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $P/p2 -o run -- python tools/deep_fwd.py > $P/p2.log 2>&1 || exit 5
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE TCC_HIT TCC_MISS --output-format csv -d $P/p3 -o run -- python tools/deep_fwd.py > $P/p3.log 2>&1 || exit 6
fi
echo done
