#!/bin/bash
# Round evidence on the GPU box, everything under gpurun_out/ (the box's
# profiles/ is not merged back; summarise locally with tools/pmc_summary.py and
# tools/wide_prof_summary.py). PART=a: -m gpu suite, smoke, profiles_run.sh +
# box-side pmc_summary (so the bench line carries roofline.traffic), frame
# timeline, the default bench line. PART=b: config 2 and config 5 bench lines,
# the wide gather's stats + PMC, the per-rank N = 2 / 4 / 8 projection.
set -u
cd ${GRAFT_REPO_ROOT:-.}
TAG=${1:-r04x}
mkdir -p gpurun_out
if [ "${PART:-a}" = a ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=25 > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_tests.log; exit 1; }
  tail -1 gpurun_out/gpu_tests.log
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 gpurun_out/smoke.log; exit 2; }
  tail -1 gpurun_out/smoke.log
  bash profiles_run.sh $TAG || { echo PROFILE_FAILED; exit 4; }
  python3 tools/pmc_summary.py $TAG > gpurun_out/pmc_summary.log 2>&1 || { tail gpurun_out/pmc_summary.log; exit 5; }
  f=$(ls gpurun_out/prof/trace/*kernel_trace.csv 2>/dev/null | head -1)
  [ -n "$f" ] && python3 tools/timeline.py $f > gpurun_out/frame_timeline.txt 2>&1
  timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/bench.log; exit 3; }
  tail -1 gpurun_out/bench.log | cut -c1-400
else
  timeout -k 10 300 python -u bench.py --config 2 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c2.log 2>&1 || { echo BENCH_C2_FAILED; tail -20 gpurun_out/bench_c2.log; exit 6; }
  tail -1 gpurun_out/bench_c2.log | cut -c1-300
  timeout -k 10 300 python -u bench.py --config 5 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c5.log 2>&1 || { echo BENCH_C5_FAILED; tail -20 gpurun_out/bench_c5.log; exit 7; }
  tail -1 gpurun_out/bench_c5.log | cut -c1-300
  LIB=lib bash tools/gpu_wide_prof.sh || exit 8
  # per-rank cost at N = 2 / 4 / 8 on this one GPU, every rank
  WORLDS="2 4 8" timeout -k 10 900 python -u tools/rank_projection.py > gpurun_out/rank_projection.jsonl 2> gpurun_out/rank_projection_ranks.log || { echo PROJ_FAILED; tail -20 gpurun_out/rank_projection_ranks.log; exit 9; }
  cat gpurun_out/rank_projection.jsonl | cut -c1-300
fi
echo final-done
