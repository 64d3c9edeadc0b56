#!/bin/bash
# config 5's k = 200 caustic gather per library: isolated (tools/wide_probe.py)
# and in the config-5 frame pipeline (tools/ab_frame.py --scene caustics).
set -u
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out/wide
for v in ${LIBS:-lib}; do
  PM_HIP_LIB=photon-mapping_amd/$v/libpm_hip.so timeout -k 10 200 python -u tools/wide_probe.py --frames 4 > gpurun_out/wide/$v.probe.log 2>&1 || { echo "PROBE_FAILED $v"; tail -5 gpurun_out/wide/$v.probe.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/wide/$v.probe.log)"
done
if [ "${FRAME:-1}" = 1 ]; then
  LIBS="${LIBS:-lib}" REPS=${REPS:-1} AB_ARGS="--scene caustics --caustic 6250000 --caustic-k 200 --steps 2" bash tools/ab_libs.sh || exit $?
fi
echo wide-done
