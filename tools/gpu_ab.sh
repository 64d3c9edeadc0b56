#!/bin/bash
# A/B bench lines per library variant: tools/gpu_ab.sh "<bench args>" lib lib_x ...
set -u
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
ARGS=$1; shift
mkdir -p gpurun_out/ab
for v in "$@"; do
  L=$R/photon-mapping_amd/$v/libpm_hip.so
  [ -f $L ] || { echo "no $v"; continue; }
  tag=$(echo "$v $ARGS" | tr -c 'a-zA-Z0-9_\n' '_')
  PM_HIP_LIB=$L timeout -k 10 300 python -u bench.py $ARGS --no-cpu-baseline --no-secondary > gpurun_out/ab/$tag.log 2>&1 || { echo AB_FAILED $v; tail -20 gpurun_out/ab/$tag.log; exit 1; }
  python3 -c "
import json,sys
d=json.loads(open('gpurun_out/ab/$tag.log').read().strip().splitlines()[-1])
print('$v', '$ARGS', 'ms/frame', d['ms_per_frame'], 'phases', {k: round(v,2) for k,v in d['phases_ms'].items()})"
done
