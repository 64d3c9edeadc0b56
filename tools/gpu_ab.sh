# A/B helper: GPU tests, then traversal + bench for the default library and an
# optional variant (VARIANT=lib_xxx), all outputs under gpurun_out/.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 200 python tools/trav_bench.py > gpurun_out/trav_default.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 > gpurun_out/bench_default.log 2>&1
for v in $VARIANTS; do
  PM_HIP_LIB=photon-mapping_amd/$v/libpm_hip.so timeout -k 10 200 python tools/trav_bench.py > gpurun_out/trav_$v.log 2>&1
  PM_HIP_LIB=photon-mapping_amd/$v/libpm_hip.so timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 > gpurun_out/bench_$v.log 2>&1
done
