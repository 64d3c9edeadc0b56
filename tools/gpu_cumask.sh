#!/bin/bash
# CU-masked render side stream A/B (tools/cumask_probe.py), config 3 bench frames.
set -u
mkdir -p gpurun_out/cm
for rep in 1 2; do
  for m in none 0x77777777 0x55555555 0x3f3f3f3f; do
    timeout -k 10 200 python -u tools/cumask_probe.py $m -- --steps 5 --warmup 3 --no-cpu-baseline --no-secondary > gpurun_out/cm/b.log 2>&1 || { tail gpurun_out/cm/b.log; exit 2; }
    python - "$m" <<'PY'
import json, sys
line = [l for l in open("gpurun_out/cm/b.log") if l.startswith("{")][-1]
d = json.loads(line)
p = d["phases_ms"]
print(f"{sys.argv[1]:12s} frame {d['ms_per_frame']:8.2f} " + " ".join(f"{k} {v:6.2f}" for k, v in p.items() if k != "exchange"), flush=True)
PY
  done
done
