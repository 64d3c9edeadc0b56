set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "kdtree or check_variant or sharded or workloads or golden or knn" > gpurun_out/kd_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/kd_tests.log; exit 1; }
tail -3 gpurun_out/kd_tests.log
LIBS="lib_old lib" REPS=2 bash tools/ab_libs.sh
