#!/bin/bash
# Kernel trace + separate PMC passes of the isolated wide-gather probe.
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/probe_prof
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
P="python3 $R/tools/wide_probe.py --frames 2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o p -- $P > $OUT/trace.log 2>&1 || { echo TRACE_FAILED; tail $OUT/trace.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o p -- $P > $OUT/fetch.log 2>&1 || { echo FETCH_FAILED; exit 2; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o p -- $P > $OUT/write.log 2>&1 || { echo WRITE_FAILED; exit 3; }
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $OUT/sq -o p -- $P > $OUT/sq.log 2>&1 || { echo SQ_FAILED; exit 4; }
echo probe-prof-done
