#!/bin/bash
# round 5 (r05r): counters of the current configs[2] forward (deep_conv3_kernel<20> with its
# LDS-DMA ring, deep_front_kernel), then the headline bench + rocprof kernel stats of the loop
set -o pipefail
REPS=3 bash tools/pmc_any.sh r05r_pmc_deep tools/deep_fwd.py || exit 1
bash tools/prof_headline.sh r05r_h || exit 2
echo done
