#!/bin/bash
# Wide-gather (k > 64) check on the GPU box: parity tests for k != 50, the
# config-5 bench line, walk statistics of the stats variants (lib_ws: subtree
# boxes, lib_wsn: plane test only) and a kernel-trace profile.
set -u
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
TAG=${1:-r03x}
mkdir -p gpurun_out/prof_c5
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "tests/test_gpu_parity.py::test_gather_k_vs_oracle" tests/test_gpu_parity.py::test_render_caustic_k200_vs_oracle \
  tests/test_gpu_workloads.py::test_config5_caustics_reduced tests/test_gpu_fullsize.py::test_config5_full_size_vs_oracle \
  > gpurun_out/wide_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/wide_tests.log; exit 1; }
tail -3 gpurun_out/wide_tests.log
timeout -k 10 300 python -u bench.py --config 5 --steps 5 --warmup 2 --no-cpu-baseline --no-secondary > gpurun_out/bench_c5.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/bench_c5.log; exit 3; }
tail -1 gpurun_out/bench_c5.log
for v in ws wsn; do
  [ -f photon-mapping_amd/lib_$v/libpm_hip.so ] || continue
  PM_HIP_LIB=$R/photon-mapping_amd/lib_$v/libpm_hip.so timeout -k 10 300 python -u bench.py --config 5 --steps 1 --warmup 0 --no-cpu-baseline --no-secondary > gpurun_out/stats_$v.log 2>&1 || { echo STATS_FAILED $v; tail -20 gpurun_out/stats_$v.log; exit 5; }
  grep "\[wide" gpurun_out/stats_$v.log | tail -2
done
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c5 -o $TAG -- python3 $R/bench.py --config 5 --steps 2 --warmup 1 --no-cpu-baseline --no-secondary > $R/gpurun_out/prof_c5/trace.log 2>&1 || { echo PROF_FAILED; exit 4; }
echo wide-done
