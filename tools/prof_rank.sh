#!/bin/bash
# Kernel-trace stats of replayed N-rank frames (tools/rank_projection.py) on the
# GPU box: WORLDS / RANKS / REPS as that tool takes them -> gpurun_out/prof_<tag>/
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-rank}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o $TAG -- python3 $R/tools/rank_projection.py > $OUT/run.log 2>&1 || { tail -20 $OUT/run.log; exit 1; }
f=$(find $OUT -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:45]:
    print(f'{r["Name"].split("(")[0][:70]:70s} calls={int(r["Calls"]):5d} total_ms={float(r["TotalDurationNs"])/1e6:8.2f} avg_us={float(r["AverageNs"])/1e3:9.1f}')
PY
