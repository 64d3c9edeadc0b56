#!/bin/bash
# Kernel-trace stats of bench.py (config 3, N = 1) for each library of $LIBS
# (GPU box, repo root): the top kernels per library side by side.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
for v in $LIBS; do
  OUT=$R/gpurun_out/prof_lib_$v
  mkdir -p $OUT
  (cd /tmp && PM_HIP_LIB=$R/photon-mapping_amd/$v/libpm_hip.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o s -- python3 $R/bench.py --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --no-secondary ${BENCH_ARGS:-} > $OUT/run.log 2>&1) || { tail -20 $OUT/run.log; exit 1; }
done
python3 - $LIBS <<'PY'
import csv, glob, sys, os
R = os.environ.get("GRAFT_REPO_ROOT", os.getcwd())
tabs = {}
for v in sys.argv[1:]:
    f = glob.glob(f"{R}/gpurun_out/prof_lib_{v}/**/*kernel_stats.csv", recursive=True)[0]
    tabs[v] = {r["Name"].split("(")[0][:60]: (int(r["Calls"]), float(r["TotalDurationNs"]) / 1e6) for r in csv.DictReader(open(f))}
first = tabs[sys.argv[1]]
for k in sorted(first, key=lambda k: -first[k][1])[:30]:
    print(f"{k:60s} " + " ".join(f"{v}: {tabs[v].get(k, (0, 0.0))[1]:8.2f}" for v in sys.argv[1:]))
PY
