# Gather-kernel diagnostics: walk/insert stats, then SQ counters (separate PMC pass).
set -e
R=$(pwd); export TMPDIR=/tmp; mkdir -p gpurun_out/pg
PM_GATHER_STATS=1 timeout -k 10 300 python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-secondary > gpurun_out/pg/stats.log 2>&1
cd /tmp
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD --output-format csv -d $R/gpurun_out/pg/pmc -o g -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-secondary > $R/gpurun_out/pg/pmc.log 2>&1
