#!/bin/bash
# Config 5's k = 200 caustic gather alone (tools/wide_probe.py) under rocprofv3:
# kernel-trace stats, then separate PMC passes (HBM bytes, wave occupancy and
# waiting). Summarise with tools/wide_prof_summary.py <tag>.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
V=${LIB:-lib}
OUT=$R/gpurun_out/wide_prof/$V
mkdir -p $OUT
export PM_HIP_LIB=$R/photon-mapping_amd/$V/libpm_hip.so
export TMPDIR=/tmp
cd /tmp
P="python3 $R/tools/wide_probe.py --frames ${FRAMES:-2}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o wide -- $P > $OUT/trace.log 2>&1 || { echo WIDE_TRACE_FAILED; tail -5 $OUT/trace.log; exit 1; }
[ "${PMC:-1}" = 1 ] || { echo wide-prof-done; exit 0; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o wide -- $P > $OUT/fetch.log 2>&1 || { echo WIDE_FETCH_FAILED; exit 2; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o wide -- $P > $OUT/write.log 2>&1 || { echo WIDE_WRITE_FAILED; exit 3; }
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU --output-format csv -d $OUT/pmc_sq -o wide -- $P > $OUT/sq.log 2>&1 || { echo WIDE_SQ_FAILED; exit 4; }
echo wide-prof-done
