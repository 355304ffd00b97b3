cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_bson.py tests/test_qnet_gpu.py -q --timeout 200 --timeout-method thread -k "bson or episode_schedule or load_trainer" 2>&1 | tail -15
