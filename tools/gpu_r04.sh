#!/bin/bash
# Round-4 GPU call: the -m gpu suite, then an A/B of variant libraries
# (LIBS) on the config-3 frame. Stops at the first fault / abort / timeout.
set -u
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 ${TEST_TIMEOUT:-700} python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    --durations=25 ${TEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1
  rc=$?
  tail -25 gpurun_out/gpu_tests.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "TESTS_RC=$rc: stopping"; exit $rc; fi
  echo "TESTS_RC=$rc"
fi
if [ -n "${LIBS:-}" ]; then
  LIBS="$LIBS" REPS=${REPS:-2} AB_ARGS="${AB_ARGS:-}" bash tools/ab_libs.sh || exit $?
fi
if [ "${BENCH:-0}" = 1 ]; then
  timeout -k 10 400 python -u bench.py ${BENCH_ARGS:---steps 10 --warmup 3} > gpurun_out/bench.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/bench.log; exit 3; }
  tail -1 gpurun_out/bench.log
fi
echo call-done
