# round 4: the dense_h3 forward test with its h3-vs-x6 spread printed
set -o pipefail
OUT=gpurun_out/r04zh; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread tests/test_qnet_gpu.py -k dense_h3 -m gpu > $OUT/t.log 2>&1; rc=$?
grep -h "dense_h3 vs x6\|passed\|failed" $OUT/t.log; [ $rc -eq 0 ] || exit 1
echo done
