#!/bin/bash
# Issue-side PMC passes (GPU box, repo root): instruction mix, VALU activity and
# lane utilisation of every kernel of one bench frame. Summarised by
# tools/pmc_issue.py. Each pass is its own run (no trace domains with --pmc).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/issue
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES --output-format csv -d $OUT/a -o a -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-secondary > $OUT/a.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_BRANCH SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_CYCLES SQ_WAVES --output-format csv -d $OUT/b -o b -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-secondary > $OUT/b.log 2>&1 || exit 2
cd $R && python3 tools/pmc_issue.py
