#!/bin/bash
# A/B of the bounce-ray sort knobs on config 3 (run on the GPU box from the repo root).
set -e
mkdir -p gpurun_out/tsort
for v in "PM_TRACE_SORT=0" "PM_TRACE_SORT_BITS=24" "PM_TRACE_SORT_BITS=16" "PM_TRACE_SORT_BITS=12"; do
  env $v timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 > gpurun_out/tsort/b.log 2>&1
  python - "$v" <<'PY'
import json, sys
line = [l for l in open("gpurun_out/tsort/b.log") if l.startswith("{")][-1]
d = json.loads(line)
print(f"{sys.argv[1]:45s} frame {d['ms_per_frame']:8.2f} ms  trace {d['phases_ms']['trace']:7.2f} ms")
PY
done
