#!/bin/bash
# update-path launches unpaired (each half of a paired launch on its own): bash tools/unpair2.sh <tag>
set -o pipefail
TAG=${1:-up}
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
SNK_UNPAIR=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-dbuild --no-extras > $OUT/pb.json 2> $OUT/prof.err || exit 3
python - "$OUT/prof" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:30]:
    print(f'{float(r["AverageNs"])/1e3:9.1f} us  x{r["Calls"]:>6}  {r["Name"][:150]}')
PY
