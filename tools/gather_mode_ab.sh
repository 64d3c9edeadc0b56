#!/bin/bash
# A/B of PM_GATHER_MODE on config 3 (GPU box, repo root): frame and global-gather ms.
set -e
mkdir -p gpurun_out/gmode
for v in ${MODES:-9 11 9 11}; do
  PM_GATHER_MODE=$v timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 > gpurun_out/gmode/b.log 2>&1
  python - "$v" <<'PY'
import json, sys
line = [l for l in open("gpurun_out/gmode/b.log") if l.startswith("{")][-1]
d = json.loads(line)
print(f"mode {sys.argv[1]:4s} frame {d['ms_per_frame']:8.2f}  gather_global {d['phases_ms']['gather_global']:7.2f}  gather {d['phases_ms']['gather']:7.2f}")
PY
done
