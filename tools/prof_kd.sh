# kd-build focused: GPU kd/kNN tests, then one rocprof'd bench frame
set -e
R=$(pwd); export TMPDIR=/tmp; mkdir -p gpurun_out/pkd
timeout -k 10 600 python -m pytest tests -m gpu -x -q -k "kdtree or knn or gather or render or export" > gpurun_out/pkd/pytest.log 2>&1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pkd/a -o a -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-secondary > $R/gpurun_out/pkd/a.log 2>&1
