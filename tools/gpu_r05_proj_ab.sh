#!/bin/bash
# Replayed N-rank frames (tools/rank_projection.py) for each library of $LIBS,
# alternating, $REPS rounds (GPU box, repo root). WORLDS / RANKS as the tool.
set -u
mkdir -p gpurun_out/ab
for rep in $(seq ${REPS:-2}); do
  for v in $LIBS; do
    PM_HIP_LIB=photon-mapping_amd/$v/libpm_hip.so WORLDS=${WORLDS:-8} RANKS="${RANKS:-2}" REPS=3 timeout -k 10 200 python tools/rank_projection.py > gpurun_out/ab/p.log 2> gpurun_out/ab/p.err || { tail gpurun_out/ab/p.err; exit 3; }
    python - "$v" <<'PY'
import json, sys
for l in open("gpurun_out/ab/p.log"):
    d = json.loads(l)
    print(f"{sys.argv[1]:10s} N={d['world']} ranks {d['rank_frame_ms']} slowest {d['slowest_phases_ms']}", flush=True)
PY
  done
done
