#!/bin/bash
# A/B of library variants on the GPU box (repo root):
#   TESTS="tests/test_gpu_parity.py ..." REPS=2 ARGS="--config 3" bash tools/ab.sh lib lib_x lib@--frame-opt,x=0 ...
# 1. the GPU tests named in $TESTS (none: skipped) on the production library;
# 2. $REPS alternating rounds of `bench.py $ARGS --steps 3` per entry, one line
#    each: ms/frame + phases. An entry is a library directory
#    (photon-mapping_amd/<v>/libpm_hip.so), optionally @ extra bench arguments
#    (commas for spaces).
set -u
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out/ab
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-500} python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/ab/tests.log 2>&1 || { tail -40 gpurun_out/ab/tests.log; exit 1; }
  tail -1 gpurun_out/ab/tests.log
fi
# STATS="regex": instead of the bench lines, each entry's rocprofv3 --kernel-trace
# --stats of `bench.py $ARGS --steps 2 --warmup 1`: ms per frame of the kernels
# whose names match
if [ -n "${STATS:-}" ]; then
  export TMPDIR=/tmp
  R=$(pwd)
  for e in "$@"; do
    v=${e%%@*}
    X=""
    [ "$e" != "$v" ] && X=$(echo "${e#*@}" | tr ',' ' ')
    tag=$(echo "$e" | tr -c 'a-zA-Z0-9_\n' '_')
    (cd /tmp && PM_HIP_LIB=$R/photon-mapping_amd/$v/libpm_hip.so timeout -k 10 300 rocprofv3 --kernel-trace --stats \
      --output-format csv -d $R/gpurun_out/ab/st_$tag -o s -- python3 $R/bench.py ${ARGS:-} $X --steps 2 --warmup 1 \
      --no-cpu-baseline --no-secondary > $R/gpurun_out/ab/st_$tag.log 2>&1) || { echo "STATS_FAILED $e"; exit 4; }
    python3 - "$e" "$(ls gpurun_out/ab/st_$tag/*/s_kernel_stats.csv gpurun_out/ab/st_$tag/s_kernel_stats.csv 2>/dev/null | head -1)" "$STATS" <<'PY'
import csv, re, sys
e, f, pat = sys.argv[1:4]
for r in csv.DictReader(open(f)):
    if re.search(pat, r["Name"]):
        print(f"{e:28s} {r['Name'][:60]:60s} calls {r['Calls']:>4s} ms/frame {float(r['TotalDurationNs']) / 3e6:8.3f}", flush=True)
PY
  done
  exit 0
fi
for rep in $(seq ${REPS:-2}); do
  for e in "$@"; do
    v=${e%%@*}
    X=""
    [ "$e" != "$v" ] && X=$(echo "${e#*@}" | tr ',' ' ')
    L=photon-mapping_amd/$v/libpm_hip.so
    [ -f $L ] || { echo "no $L"; exit 3; }
    tag=$(echo "$e" | tr -c 'a-zA-Z0-9_\n' '_')
    PM_HIP_LIB=$L timeout -k 10 300 python -u bench.py ${ARGS:-} $X --steps ${STEPS:-3} --no-cpu-baseline --no-secondary \
      > gpurun_out/ab/b_$tag.log 2>&1 || { echo "AB_FAILED $e"; tail -20 gpurun_out/ab/b_$tag.log; exit 2; }
    python3 - "$e" "$tag" <<'PY'
import json, sys
e, tag = sys.argv[1], sys.argv[2]
d = json.loads([l for l in open(f"gpurun_out/ab/b_{tag}.log") if l.startswith("{")][-1])
p = d["phases_ms"]
print(f"{e:28s} frame {d['ms_per_frame']:8.2f} " + " ".join(f"{k} {x:6.2f}" for k, x in p.items() if k != "exchange")
      + f" traced/s {d.get('mphotons_traced_per_s')}", flush=True)
PY
  done
done
