cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_dist_gpu.py -q --timeout 200 --timeout-method thread 2>&1 | tail -3
