#!/bin/bash
# A/B of PM_SEED_LEVELS (leader strides of the seeded gather) on config 3 (GPU box,
# repo root): frame and global-gather ms. Runs the seeded-gather bitwise tests first.
set -u
mkdir -p gpurun_out/seed
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "seeded or modes" -x -q --timeout 120 --timeout-method thread > gpurun_out/seed/tests.log 2>&1 || { tail -30 gpurun_out/seed/tests.log; exit 1; }
tail -2 gpurun_out/seed/tests.log
for v in ${LEVELS:-16 256,16 128,16 512,32 4096,256,16 16}; do
  PM_SEED_LEVELS=$v timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 > gpurun_out/seed/b.log 2>&1 || { tail gpurun_out/seed/b.log; exit 2; }
  python - "$v" <<'PY'
import json, sys
line = [l for l in open("gpurun_out/seed/b.log") if l.startswith("{")][-1]
d = json.loads(line)
print(f"levels {sys.argv[1]:14s} frame {d['ms_per_frame']:8.2f}  gather_global {d['phases_ms']['gather_global']:7.2f}  gather {d['phases_ms']['gather']:7.2f}", flush=True)
PY
done
