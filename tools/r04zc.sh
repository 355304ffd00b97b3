# round 4: final: full GPU suite + the driver bench command
set -o pipefail
OUT=gpurun_out/r04zc; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $OUT/t.log 2>&1; rc=$?
tail -n 2 $OUT/t.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/b20.json 2> $OUT/b20.err || exit 2
python -c "import json; d=json.load(open('$OUT/b20.json')); print(d['value'], d['ms_per_step'], d['d_build_sec'], d['configs2']['value'], d['reference_ratio']['updates_per_s'], d['laplace_sampling']['seconds'], d['configs3_per_rank']['value'])"
echo done
