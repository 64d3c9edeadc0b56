#!/bin/bash
# Fused photon paths (PM_TRACE_FUSED) A/B on the GPU box: config-3 bench frames
# per (library, frame options) of $RUNS ("lib:opt1,opt2" or "lib:-"), $REPS rounds.
set -u
mkdir -p gpurun_out/ab
for rep in $(seq ${REPS:-1}); do
  for run in $RUNS; do
    v=${run%%:*}; o=${run#*:}
    args=""
    [ "$o" != "-" ] && for x in ${o//,/ }; do args="$args --frame-opt $x"; done
    PM_HIP_LIB=photon-mapping_amd/$v/libpm_hip.so timeout -k 10 200 python bench.py --config ${CONFIG:-3} --no-cpu-baseline --no-secondary --steps ${STEPS:-5} $args > gpurun_out/ab/f.log 2>&1 || { tail gpurun_out/ab/f.log; exit 2; }
    python - "$v" "$o" <<'PY'
import json, sys
d = json.loads([l for l in open("gpurun_out/ab/f.log") if l.startswith("{")][-1])
p = d["phases_ms"]
print(f"{sys.argv[1]:10s} {sys.argv[2]:22s} frame {d['ms_per_frame']:8.2f} " + " ".join(f"{k} {v:6.2f}" for k, v in p.items() if k != "exchange"), flush=True)
PY
  done
done
