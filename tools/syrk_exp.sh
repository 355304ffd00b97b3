cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_laplace_gpu.py -q --timeout 200 --timeout-method thread -k "gram" 2>&1 | tail -2
timeout -k 10 200 python tools/dbuild.py 50000 2 2>&1 | tail -1
