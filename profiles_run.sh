#!/bin/bash
# Profiling recipe (run on the GPU box from the repo root): kernel-trace stats of
# the bench command, then separate PMC passes (never combined with trace domains).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof
TAG=${1:-r01}
ARGS=${BENCH_ARGS:---steps 2 --warmup 1 --no-cpu-baseline --no-secondary}
mkdir -p $OUT
sha256sum $R/photon-mapping_amd/lib/libpm_hip.so > $OUT/lib.sha256
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o $TAG -- python3 $R/bench.py $ARGS > $OUT/${TAG}_trace_bench.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o $TAG -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-secondary > $OUT/${TAG}_fetch.log 2>&1 || exit 2
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o $TAG -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-secondary > $OUT/${TAG}_write.log 2>&1 || exit 3
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/pmc_sq -o $TAG -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-secondary > $OUT/${TAG}_sq.log 2>&1 || exit 4
echo profile-done
