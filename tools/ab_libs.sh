#!/bin/bash
# A/B of variant libraries on the GPU box: tools/ab_frame.py for each library
# of $LIBS (photon-mapping_amd/<dir>), $REPS rounds alternating; every variant
# must print the same image digest. Output: gpurun_out/ab/ab.jsonl
set -u
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out/ab
: > gpurun_out/ab/ab.jsonl
for rep in $(seq ${REPS:-2}); do
  for v in $LIBS; do
    PM_HIP_LIB=photon-mapping_amd/$v/libpm_hip.so timeout -k 10 200 python -u tools/ab_frame.py ${AB_ARGS:-} >> gpurun_out/ab/ab.jsonl 2> gpurun_out/ab/err.log || { tail -20 gpurun_out/ab/err.log; exit 1; }
    tail -1 gpurun_out/ab/ab.jsonl
  done
done
python3 - <<'PY'
import json
rows = [json.loads(l) for l in open("gpurun_out/ab/ab.jsonl")]
digs = {json.dumps(r["digest"]) for r in rows}
print("image digests identical across variants:", len(digs) == 1)
PY
