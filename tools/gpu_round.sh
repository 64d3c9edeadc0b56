#!/bin/bash
# Round evidence on the GPU box (repo root): full -m gpu suite, smoke, the
# driver's bench command, then profiles_run.sh (kernel-trace stats + separate
# PMC passes) summarised by tools/pmc_summary.py into profiles/<tag>_*.
set -u
cd $GRAFT_REPO_ROOT
TAG=${1:-r02x}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread --durations=15 > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 gpurun_out/smoke.log; exit 2; }
tail -1 gpurun_out/smoke.log
# counters first: pmc_summary writes profiles/pmc_gather_global.json for THIS
# library, so the bench line below (and the driver's, on the same library)
# carries roofline.traffic
bash profiles_run.sh $TAG || { echo PROFILE_FAILED $?; exit 4; }
python3 tools/pmc_summary.py $TAG > gpurun_out/pmc_summary.log 2>&1 || { tail gpurun_out/pmc_summary.log; exit 5; }
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/bench.log; exit 3; }
tail -1 gpurun_out/bench.log
timeout -k 10 300 python -u bench.py --config 2 --steps 10 --warmup 3 > gpurun_out/bench_c2.log 2>&1 || { echo BENCH_C2_FAILED; tail -20 gpurun_out/bench_c2.log; exit 6; }
tail -1 gpurun_out/bench_c2.log
timeout -k 10 300 python -u bench.py --config 5 --steps 5 --warmup 2 > gpurun_out/bench_c5.log 2>&1 || { echo BENCH_C5_FAILED; tail -20 gpurun_out/bench_c5.log; exit 7; }
tail -1 gpurun_out/bench_c5.log
cp gpurun_out/gpu_tests.log profiles/${TAG}_gpu_tests.log
cp gpurun_out/bench.log profiles/${TAG}_bench.json.log
cp gpurun_out/bench_c2.log profiles/${TAG}_bench_config2.json.log
echo round-done
