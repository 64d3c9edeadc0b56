#!/bin/bash
# Gather experiment round (GPU box, repo root): gather parity tests, mode A/B,
# then kernel-trace stats of the diagnostic modes in $DIAG (per-kernel split).
set -u
mkdir -p gpurun_out/gexp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gather or knn" > gpurun_out/gexp/t.log 2>&1 || { tail -30 gpurun_out/gexp/t.log; exit 1; }
tail -2 gpurun_out/gexp/t.log
MODES="${MODES:-12 13}" bash tools/gather_mode_ab.sh || exit 2
export TMPDIR=/tmp
for d in ${DIAG:-}; do
  (cd /tmp && PM_GATHER_MODE=$d timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/gexp/p$d -o m$d -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/gexp/p$d.log 2>&1) || exit 3
  python3 - "$d" <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/gexp/p{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "gather" in r["Name"]:
        print(sys.argv[1], r["Name"][:90], r["Calls"], float(r["AverageNs"]) / 1e6)
PY
done
