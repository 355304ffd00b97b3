# round 4: counter passes for the act forward (conv_h3f after the prologue change, dense_h3) and the
# B = 64 update kernels (train_iter.py), each counter set in its own rocprofv3 run
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/pmc_traffic.sh r04z h3f || exit 1
bash tools/pmc_any.sh r04z_act tools/act_fwd.py || exit 2
ITERS=16 bash tools/pmc_any.sh r04z_upd tools/train_iter.py || exit 3
U=gpurun_out/r04z_upd
ITERS=16 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE TCC_HIT TCC_MISS --output-format csv -d $U/p3 -o run -- python tools/train_iter.py > $U/p3.log 2>&1 || exit 4
echo done
