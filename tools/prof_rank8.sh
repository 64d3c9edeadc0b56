#!/bin/bash
# Kernel trace of one replayed N = 8 rank frame (rank ${RANK:-0}, second of two),
# GPU box, repo root: gpurun_out/rank8_timeline.txt (tools/timeline.py).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
OUT=$R/gpurun_out/prof_rank8
mkdir -p $OUT
(cd /tmp && WORLDS=8 RANKS=${RANK:-0} REPS=2 timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o s -- python3 $R/tools/rank_projection.py > $OUT/run.log 2>&1) || { tail -20 $OUT/run.log; exit 1; }
f=$(ls $OUT/*kernel_trace.csv $OUT/*/*kernel_trace.csv 2>/dev/null | head -1)
python3 $R/tools/timeline.py $f > $R/gpurun_out/rank8_timeline.txt 2>&1
head -80 $R/gpurun_out/rank8_timeline.txt
