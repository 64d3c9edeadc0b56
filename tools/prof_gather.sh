#!/bin/bash
# PMC passes over tools/gather_sweep.py (mode 0) for the gather kernels.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/profg
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
rocprofv3 -L > $OUT/counters.txt 2>&1 || true
P="python3 $R/tools/gather_sweep.py PM_GATHER_MODE=0"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD --output-format csv -d $OUT/p1 -o g -- $P > $OUT/p1.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/p2 -o g -- $P > $OUT/p2.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD --output-format csv -d $OUT/p3 -o g -- $P > $OUT/p3.log 2>&1 || exit 3
echo done
