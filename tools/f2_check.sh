cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_laplace_gpu.py -q --timeout 300 --timeout-method thread -k "normals or sample_model or sampling" 2>&1 | tail -3
timeout -k 10 300 python tools/lap_sampling.py 5000 12 2>&1 | tail -1
