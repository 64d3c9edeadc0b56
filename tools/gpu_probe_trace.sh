#!/bin/bash
# Kernel trace of the isolated wide-gather probe per library variant.
set -u
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp
for v in "$@"; do
  OUT=$R/gpurun_out/probe_trace_$v
  mkdir -p $OUT
  PM_HIP_LIB=$R/photon-mapping_amd/$v/libpm_hip.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o p -- python3 $R/tools/wide_probe.py --frames 2 > $OUT/log 2>&1 || { echo TRACE_FAILED $v; tail $OUT/log; exit 1; }
  echo "== $v"; grep "gather ms" $OUT/log; grep -h "gather_wide" $OUT/p_kernel_stats.csv | cut -d, -f1-4 | cut -c1-60,200-
done
