#!/bin/bash
# Round-5 A/B on the GPU box (repo root): for each library of $LIBS
# (photon-mapping_amd/<dir>), alternating, $REPS rounds: config 3 and config 2
# bench lines (N = 1) and the replayed N = 8 rank frames (tools/rank_projection.py).
set -u
mkdir -p gpurun_out/ab
for rep in $(seq ${REPS:-2}); do
  for v in $LIBS; do
    export PM_HIP_LIB=photon-mapping_amd/$v/libpm_hip.so
    for c in ${CONFIGS:-3 2}; do
      timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --no-secondary --steps ${STEPS:-5} > gpurun_out/ab/b.log 2>&1 || { tail gpurun_out/ab/b.log; exit 2; }
      python - "$v" "$c" <<'PY'
import json, sys
d = json.loads([l for l in open("gpurun_out/ab/b.log") if l.startswith("{")][-1])
p = d["phases_ms"]
print(f"{sys.argv[1]:12s} config{sys.argv[2]} frame {d['ms_per_frame']:8.2f} " + " ".join(f"{k} {v:6.2f}" for k, v in p.items() if k != "exchange"), flush=True)
PY
    done
    if [ -n "${PROJ:-}" ]; then
      WORLDS=8 RANKS="${PROJ_RANKS:-0 2}" timeout -k 10 200 python tools/rank_projection.py > gpurun_out/ab/p.log 2> gpurun_out/ab/p.err || { tail gpurun_out/ab/p.err; exit 3; }
      python - "$v" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab/p.log").readline())
print(f"{sys.argv[1]:12s} N=8 ranks {d['rank_frame_ms']} slowest {d['slowest_phases_ms']}", flush=True)
PY
    fi
  done
done
