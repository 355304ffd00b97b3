# round 4: lap_act_kernel rings (laplace tests + the 5000-model timing + kernel stats)
set -o pipefail
OUT=gpurun_out/r04c; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_laplace_gpu.py -m gpu > $OUT/t.log 2>&1; rc=$?
tail -n 3 $OUT/t.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python tools/lap_sampling.py > $OUT/ls.json 2>&1 || exit 2
cat $OUT/ls.json | tail -3
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python tools/lap_sampling.py > $OUT/ls_prof.json 2>&1 || exit 3
python tools/kstats.py $OUT/prof | head -12
echo done
