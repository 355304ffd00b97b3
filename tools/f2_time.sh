cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/lap_sampling.py 5000 12 2>&1 | tail -2
