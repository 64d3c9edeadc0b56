# A/B helper: bench (no CPU baseline) for the default build and each entry of
# $VARIANTS: "lib_xxx" (photon-mapping_amd/lib_xxx/libpm_hip.so) or
# "env:NAME=VAL[,NAME=VAL]" (environment knobs). Outputs in gpurun_out/.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 > gpurun_out/bench_default.log 2>&1
for v in $VARIANTS; do
  tag=$(echo "$v" | tr ':=,' '___')
  if [[ $v == env:* ]]; then
    (export $(echo "${v#env:}" | tr ',' ' ') && timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 > gpurun_out/bench_$tag.log 2>&1)
  else
    PM_HIP_LIB=photon-mapping_amd/$v/libpm_hip.so timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 > gpurun_out/bench_$tag.log 2>&1
  fi
done
