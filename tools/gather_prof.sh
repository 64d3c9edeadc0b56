#!/bin/bash
# Kernel-trace stats of the gather kernels for each PM_GATHER_MODE in $DIAG (GPU box, repo root).
set -u
mkdir -p gpurun_out/gexp
export TMPDIR=/tmp
for d in ${DIAG:-13}; do
  (cd /tmp && PM_GATHER_MODE=$d timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/gexp/p$d -o m$d -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-secondary > $GRAFT_REPO_ROOT/gpurun_out/gexp/p$d.log 2>&1) || exit 3
  python3 - "$d" <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/gexp/p{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if any(k in r["Name"] for k in ("gather", "lead", "union")):
        print(sys.argv[1], r["Name"][:70], r["Calls"], "avg %.3f ms" % (float(r["AverageNs"]) / 1e6), "max %.3f" % (float(r["MaxNs"]) / 1e6))
PY
done
