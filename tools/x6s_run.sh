set -o pipefail
mkdir -p gpurun_out/x6s
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -m pytest tests/test_qnet_gpu.py -x -q > gpurun_out/x6s/t.log 2>&1; rc=$?; tail -n 5 gpurun_out/x6s/t.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python bench.py --steps 300 --no-cpu-baseline --no-dbuild > gpurun_out/x6s/b.json 2> gpurun_out/x6s/b.err || exit 2
python -c "import json;d=json.load(open('gpurun_out/x6s/b.json'));print(d['value'], d['ms_per_step'], d.get('act_forward_ms'), d['roofline'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/x6s/prof -o run -- python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-dbuild --no-extras > gpurun_out/x6s/pb.json 2> gpurun_out/x6s/prof.err || exit 3
echo done
