#!/bin/bash
# A/B of build variants on config 3 (GPU box, repo root): runs the GPU parity
# tests on the default library, then bench for default and each $VARIANTS
# entry (photon-mapping_amd/<v>/libpm_hip.so), alternating, $REPS rounds.
set -u
mkdir -p gpurun_out/ab
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/tests.log 2>&1 || { tail -30 gpurun_out/ab/tests.log; exit 1; }
tail -1 gpurun_out/ab/tests.log
for rep in $(seq ${REPS:-2}); do
  for v in default $VARIANTS; do
    if [ $v = default ]; then unset PM_HIP_LIB; else export PM_HIP_LIB=photon-mapping_amd/$v/libpm_hip.so; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --steps 3 > gpurun_out/ab/b.log 2>&1 || { tail gpurun_out/ab/b.log; exit 2; }
    python - "$v" <<'PY'
import json, sys
line = [l for l in open("gpurun_out/ab/b.log") if l.startswith("{")][-1]
d = json.loads(line)
p = d["phases_ms"]
print(f"{sys.argv[1]:14s} frame {d['ms_per_frame']:8.2f} " + " ".join(f"{k} {v:6.2f}" for k, v in p.items() if k != "exchange"), flush=True)
PY
  done
done
