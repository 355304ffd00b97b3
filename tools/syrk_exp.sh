cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 python tools/dbuild.py 16384 2 2>&1 | tail -1
SNK_SYRK_PRIO=1 timeout -k 10 120 python tools/dbuild.py 16384 2 2>&1 | tail -1
SNK_SYRK_EXP_NOLOAD=1 timeout -k 10 120 python tools/dbuild.py 16384 2 2>&1 | tail -1
SNK_SYRK_ORDER=rows timeout -k 10 120 python tools/dbuild.py 16384 2 2>&1 | tail -1
