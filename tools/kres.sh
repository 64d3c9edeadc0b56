#!/bin/bash
# Per-kernel resource usage (VGPRs, AGPRs, spills, LDS, occupancy) of one source:
#   tools/kres.sh knn.hip "-DPM_GATHER50_WIDE=2" [kernel-name-regex]
set -eu
cd "$(dirname "$0")/../photon-mapping_amd"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off \
  -fhip-fp32-correctly-rounded-divide-sqrt -fno-fast-math ${2:-} -Rpass-analysis=kernel-resource-usage \
  --cuda-device-only -c csrc/$1 -o /tmp/kres.o 2>&1 | \
  grep -E "Function Name|VGPRs:|AGPRs|ScratchSize|Occupancy|LDS Size|SGPRs:" | \
  sed -e 's/.*remark: //' | paste - - - - - - - | grep -E "${3:-.}" | \
  sed -E 's/Function Name: //; s/ \[-Rpass-analysis=kernel-resource-usage\]//g' | cut -c1-400
