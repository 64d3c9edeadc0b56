#!/bin/bash
# L1/L2 request counters of one config-3 frame (tools/ab_frame.py) per library:
#   LIBS="lib lib_x" bash tools/pmc_l2.sh  -> gpurun_out/pmc_l2/<lib>/...
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
for v in ${LIBS:-lib}; do
  OUT=$R/gpurun_out/pmc_l2/$v
  mkdir -p $OUT
  cd /tmp
  PM_HIP_LIB=$R/photon-mapping_amd/$v/libpm_hip.so timeout -s KILL 180 rocprofv3 \
    --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum \
    --output-format csv -d $OUT -o l2 -- python3 $R/tools/ab_frame.py --steps 1 > $OUT/run.log 2>&1 || { echo "PMC_FAILED $v"; tail -5 $OUT/run.log; exit 1; }
  echo "pmc-done $v"
done
