#!/bin/bash
# Replayed N = $WORLDS rank frames (tools/rank_projection.py) per library of
# $LIBS, alternating, $REPS_AB rounds (GPU box, repo root).
set -u
for rep in $(seq ${REPS_AB:-1}); do
  for v in $LIBS; do
    PM_HIP_LIB=photon-mapping_amd/$v/libpm_hip.so WORLDS=${WORLDS:-8} RANKS="${RANKS:-0 2}" timeout -k 10 400 python tools/rank_projection.py > gpurun_out/pl.jsonl 2> gpurun_out/pl.err || { tail gpurun_out/pl.err; exit 2; }
    echo "== $v"; grep "^#" gpurun_out/pl.err
  done
done
