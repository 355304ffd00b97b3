# round 4: env_step at 16 envs per workgroup up to 8,192 envs (retry after the a3max fix) -- full GPU suite, bench
set -o pipefail
OUT=gpurun_out/r04zd; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $OUT/t.log 2>&1; rc=$?
tail -n 2 $OUT/t.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-dbuild --no-configs2 --no-cpu-baseline > $OUT/b.json 2> $OUT/b.err || exit 4
python -c "import json; d=json.load(open('$OUT/b.json')); print(d['value'], d['ms_per_step'], d['step_kernel'], d['reference_ratio']['updates_per_s'])"
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-dbuild --no-configs2 --no-cpu-baseline --no-configs3 > $OUT/b20.json 2> $OUT/b20.err || exit 5
python -c "import json; d=json.load(open('$OUT/b20.json')); print('steps20', d['value'], d['ms_per_step'])"
echo done
