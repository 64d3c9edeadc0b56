#!/bin/bash
# A/B bench lines over argument sets, production library:
#   tools/gpu_opt_ab.sh "<common args>" "<args A>" "<args B>" ...
set -u
cd $GRAFT_REPO_ROOT
COMMON=$1; shift
mkdir -p gpurun_out/ab
for a in "$@"; do
  tag=$(echo "opt $COMMON $a" | tr -c 'a-zA-Z0-9_\n' '_')
  timeout -k 10 300 python -u bench.py $COMMON $a --no-cpu-baseline --no-secondary > gpurun_out/ab/$tag.log 2>&1 || { echo AB_FAILED "$a"; tail -20 gpurun_out/ab/$tag.log; exit 1; }
  python3 -c "
import json
d=json.loads(open('gpurun_out/ab/$tag.log').read().strip().splitlines()[-1])
print('[$a]', 'ms/frame', d['ms_per_frame'], 'phases', {k: round(v,2) for k,v in d['phases_ms'].items()})"
done
