#!/bin/bash
# Round-4 profile call: kernel-trace stats + PMC passes (profiles_run.sh) of
# the bench command, their summaries under profiles/<tag>_*, a per-queue frame
# timeline, then the bench line (which picks up this library's PMC traffic).
set -u
cd ${GRAFT_REPO_ROOT:-.}
TAG=${1:-r04x}
bash profiles_run.sh $TAG || { echo PROFILE_FAILED; exit 4; }
python3 tools/pmc_summary.py $TAG > gpurun_out/pmc_summary.log 2>&1 || { tail gpurun_out/pmc_summary.log; exit 5; }
f=$(ls gpurun_out/prof/trace/*kernel_trace.csv 2>/dev/null | head -1)
[ -n "$f" ] && python3 tools/timeline.py $f > profiles/${TAG}_frame_timeline.txt 2>&1
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/bench.log; exit 3; }
tail -1 gpurun_out/bench.log
cp gpurun_out/bench.log profiles/${TAG}_bench.json.log
echo prof-done
