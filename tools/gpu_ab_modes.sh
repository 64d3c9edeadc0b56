#!/bin/bash
# A/B over (library variant x PM_GATHER_MODE): VARIANTS="default lib_x", MODES="13 15".
set -e
mkdir -p gpurun_out
for v in ${VARIANTS:-default}; do
  for m in ${MODES:-13}; do
    if [[ $v == default ]]; then lib=photon-mapping_amd/lib/libpm_hip.so; else lib=photon-mapping_amd/$v/libpm_hip.so; fi
    PM_HIP_LIB=$lib PM_GATHER_MODE=$m timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 > gpurun_out/bench_${v}_m$m.log 2>&1
  done
done
