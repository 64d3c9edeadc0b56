#!/bin/bash
# LDS-side PMC pass (GPU box, repo root): bank conflicts, LDS issue stalls and
# LDS instruction counts per kernel of one bench frame (its own --pmc run, no
# trace domains), after tools/pmc_issue.sh's two passes; summary by kernel.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/issue
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_BUSY_CU_CYCLES SQ_INSTS_SMEM --output-format csv -d $OUT/c -o c -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-secondary > $OUT/c.log 2>&1 || exit 1
cd $R && python3 - <<'PY'
import collections, csv, glob
tot = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob("gpurun_out/issue/c/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        tot[r["Kernel_Name"]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in sorted(tot.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))[:14]:
    w = max(1.0, d.get("SQ_WAVES", 1))
    print(k.split("(")[0][:50].ljust(50), f"lds/wave={d.get('SQ_INSTS_LDS', 0) / w:.0f} smem/wave={d.get('SQ_INSTS_SMEM', 0) / w:.0f}",
          f"wait_inst_lds={d.get('SQ_WAIT_INST_LDS', 0) / max(1, d.get('SQ_WAVE_CYCLES', 1)):.3f}",
          f"bank_conflict/active={d.get('SQ_LDS_BANK_CONFLICT', 0) / max(1, d.get('SQ_LDS_IDX_ACTIVE', 1)):.3f}")
PY
