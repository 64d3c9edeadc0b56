#!/bin/bash
# Kernel-trace timelines of one config-3 bench frame per (library, frame options)
# pair of $RUNS ("lib:opt1,opt2" or "lib:-"), GPU box, repo root.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
for run in $RUNS; do
  v=${run%%:*}; o=${run#*:}
  args=""
  [ "$o" != "-" ] && for x in ${o//,/ }; do args="$args --frame-opt $x"; done
  tag=${v}_${o//[=,]/_}
  OUT=$R/gpurun_out/tl_$tag
  mkdir -p $OUT
  (cd /tmp && PM_HIP_LIB=$R/photon-mapping_amd/$v/libpm_hip.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o s -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-secondary $args > $OUT/run.log 2>&1) || { tail -20 $OUT/run.log; exit 1; }
  f=$(ls $OUT/*kernel_trace.csv $OUT/*/*kernel_trace.csv 2>/dev/null | head -1)
  python3 $R/tools/timeline.py $f > $R/gpurun_out/timeline_$tag.txt 2>&1
  echo "== $tag"; head -40 $R/gpurun_out/timeline_$tag.txt
done
