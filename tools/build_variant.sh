#!/bin/bash
# Build an A/B variant library: tools/build_variant.sh NAME "-DMACRO=V ..." -> photon-mapping_amd/lib_NAME/libpm_hip.so
set -eu
cd "$(dirname "$0")/../photon-mapping_amd"
make -j8 BUILD=build_$1 LIB=lib_$1/libpm_hip.so "EXTRA=$2" lib_$1/libpm_hip.so > /tmp/build_$1.log 2>&1 || { tail -20 /tmp/build_$1.log; exit 1; }
echo "built lib_$1 ($2)"
