#!/bin/bash
# Walk statistics of stats variants: tools/gpu_stats.sh "<bench args>" lib_x ...
set -u
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
ARGS=$1; shift
mkdir -p gpurun_out/stats
for v in "$@"; do
  tag=$(echo "$v $ARGS" | tr -c 'a-zA-Z0-9_\n' '_')
  PM_HIP_LIB=$R/photon-mapping_amd/$v/libpm_hip.so timeout -k 10 300 python -u bench.py $ARGS --steps 1 --warmup 0 --no-cpu-baseline --no-secondary > gpurun_out/stats/$tag.log 2>&1 || { echo STATS_FAILED $v; tail -20 gpurun_out/stats/$tag.log; exit 1; }
  echo "== $v $ARGS"; grep -E "^\[(gather50|wide)" gpurun_out/stats/$tag.log | tail -8
done
