#!/bin/bash
# Isolated wide-gather timings per library variant (tools/wide_probe.py).
set -u
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in "$@"; do
  L=$R/photon-mapping_amd/$v/libpm_hip.so
  [ -f $L ] || { echo "no $v"; continue; }
  PM_HIP_LIB=$L timeout -k 10 300 python -u tools/wide_probe.py --frames 3 > gpurun_out/probe_$v.log 2>&1 || { echo PROBE_FAILED $v; tail -20 gpurun_out/probe_$v.log; exit 1; }
  echo "== $v"; grep -E "\[wide|gather ms" gpurun_out/probe_$v.log | tail -3
done
