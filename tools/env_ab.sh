#!/bin/bash
# A/B of environment knobs on config 3 (GPU box, repo root): bench for each
# entry of $ENVS ("-" = none, else NAME=VAL[,NAME=VAL]), $REPS rounds; the GPU
# parity tests run first when $TESTS is set.
set -u
mkdir -p gpurun_out/env
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread $TESTS > gpurun_out/env/tests.log 2>&1 || { tail -30 gpurun_out/env/tests.log; exit 1; }
  tail -1 gpurun_out/env/tests.log
fi
for rep in $(seq ${REPS:-2}); do
  for v in $ENVS; do
    ( if [ "$v" != "-" ]; then export $(echo "$v" | tr ',' ' '); fi
      timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 > gpurun_out/env/b.log 2>&1 ) || { tail gpurun_out/env/b.log; exit 2; }
    python - "$v" <<'PY'
import json, sys
line = [l for l in open("gpurun_out/env/b.log") if l.startswith("{")][-1]
d = json.loads(line)
p = d["phases_ms"]
print(f"{sys.argv[1]:24s} frame {d['ms_per_frame']:8.2f} " + " ".join(f"{k} {v:6.2f}" for k, v in p.items() if k != "exchange"), flush=True)
PY
  done
done
