#!/bin/bash
# A/B of FrameConfig options on the GPU box (repo root): bench.py config $CONFIGS
# with each --frame-opt set of $OPTS ("-" = defaults; sets separated by spaces,
# options inside a set by commas), alternating, $REPS rounds.
set -u
mkdir -p gpurun_out/ab
for rep in $(seq ${REPS:-2}); do
  for o in $OPTS; do
    args=""
    [ "$o" != "-" ] && for x in ${o//,/ }; do args="$args --frame-opt $x"; done
    for c in ${CONFIGS:-3}; do
      timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --no-secondary --steps ${STEPS:-5} $args > gpurun_out/ab/f.log 2>&1 || { tail gpurun_out/ab/f.log; exit 2; }
      python - "$o" "$c" <<'PY'
import json, sys
d = json.loads([l for l in open("gpurun_out/ab/f.log") if l.startswith("{")][-1])
p = d["phases_ms"]
print(f"{sys.argv[1]:24s} config{sys.argv[2]} frame {d['ms_per_frame']:8.2f} " + " ".join(f"{k} {v:6.2f}" for k, v in p.items() if k != "exchange"), flush=True)
PY
    done
  done
done
