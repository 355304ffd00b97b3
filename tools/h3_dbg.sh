#!/bin/bash
# h3s conv3 phase timestamps (SNK_H3S_DBG) + its targeted tests: bash tools/h3_dbg.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
SNK_H3S_DBG=1 REPS=2 timeout -k 10 120 python tools/act_fwd.py 2>&1 | tail -4 || exit 1
REPS=20 timeout -k 10 120 python tools/act_fwd.py 2>&1 | tail -1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_qnet_gpu.py -q --timeout 120 --timeout-method thread -k "h3s or x6s" 2>&1 | tail -3
