#!/bin/bash
# A/B of library variants on the GPU box (repo root):
#   TESTS="tests/test_gpu_parity.py ..." REPS=2 ARGS="--config 3" bash tools/ab.sh lib lib_x ...
# 1. the GPU tests named in $TESTS (none: skipped) on the production library;
# 2. $REPS alternating rounds of `bench.py $ARGS --steps 3` per library
#    (photon-mapping_amd/<v>/libpm_hip.so), one line each: ms/frame + phases.
set -u
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out/ab
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-500} python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/ab/tests.log 2>&1 || { tail -40 gpurun_out/ab/tests.log; exit 1; }
  tail -1 gpurun_out/ab/tests.log
fi
for rep in $(seq ${REPS:-2}); do
  for v in "$@"; do
    L=photon-mapping_amd/$v/libpm_hip.so
    [ -f $L ] || { echo "no $L"; exit 3; }
    PM_HIP_LIB=$L timeout -k 10 300 python -u bench.py ${ARGS:-} --steps ${STEPS:-3} --no-cpu-baseline --no-secondary \
      > gpurun_out/ab/b_$v.log 2>&1 || { echo "AB_FAILED $v"; tail -20 gpurun_out/ab/b_$v.log; exit 2; }
    python3 - "$v" <<'PY'
import json, sys
v = sys.argv[1]
d = json.loads([l for l in open(f"gpurun_out/ab/b_{v}.log") if l.startswith("{")][-1])
p = d["phases_ms"]
print(f"{v:12s} frame {d['ms_per_frame']:8.2f} " + " ".join(f"{k} {x:6.2f}" for k, x in p.items() if k != "exchange"),
      flush=True)
PY
  done
done
