# round 4: Laplace sampling (one chunk + tr.model folded in, 32 models per D pass, 50 KB lap_act)
set -o pipefail
OUT=gpurun_out/r04f; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_laplace_gpu.py -m gpu > $OUT/t.log 2>&1; rc=$?
tail -n 2 $OUT/t.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python tools/lap_sampling.py > $OUT/ls.txt 2>&1 || exit 2
tail -1 $OUT/ls.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/lstrace -o run -- python tools/lap_sampling.py > $OUT/ls_prof.txt 2>&1 || exit 3
echo done
