#!/usr/bin/env python3
"""Per-kernel issue metrics from tools/pmc_issue.sh (gpurun_out/issue/{a,b}).

SQ cycle counters are quad-cycles (MI355X_MICROARCH.md): a wave64 VALU op takes
2 cycles, so one SIMD issues at most 2 VALU ops per quad-cycle. Reported per
kernel (sum over its launches): VALU ops per wave, lane utilisation
(THREAD_CYCLES_VALU / (64 x ACTIVE_INST_VALU)), and the VALU pipe share
valu_util = INSTS_VALU x 2 cycles / (SIMD-cycles the kernel held), with
SIMD-cycles = BUSY_CU_CYCLES x 4 quad->cycles x 4 SIMDs."""
import collections, csv, glob, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tot = collections.defaultdict(lambda: collections.defaultdict(float))
for sub in ("a", "b"):
    for f in glob.glob(os.path.join(ROOT, "gpurun_out", "issue", sub, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            tot[r["Kernel_Name"]][r["Counter_Name"]] += float(r["Counter_Value"])
rows = []
for k, d in tot.items():
    if d.get("SQ_WAVE_CYCLES", 0) < 1e8:
        continue
    w = max(1.0, d.get("SQ_WAVES", 1))
    rows.append((d["SQ_WAVE_CYCLES"], k, {
        "valu_per_wave": d.get("SQ_INSTS_VALU", 0) / w,
        "vmem_per_wave": d.get("SQ_INSTS_VMEM_RD", 0) / w,
        "salu_per_wave": d.get("SQ_INSTS_SALU", 0) / w,
        "lds_per_wave": d.get("SQ_INSTS_LDS", 0) / w,
        "f64_per_wave": (d.get("SQ_INSTS_VALU_FMA_F64", 0) + d.get("SQ_INSTS_VALU_ADD_F64", 0)) / w,
        "lane_util": d.get("SQ_THREAD_CYCLES_VALU", 0) / max(1.0, 64 * d.get("SQ_ACTIVE_INST_VALU", 1)),
        "active_frac": d.get("SQ_ACTIVE_INST_ANY", 0) / max(1.0, d.get("SQ_WAVE_CYCLES", 1)),
        "wait_frac": d.get("SQ_WAIT_ANY", 0) / max(1.0, d.get("SQ_WAVE_CYCLES", 1)),
        "wait_inst_frac": d.get("SQ_WAIT_INST_ANY", 0) / max(1.0, d.get("SQ_WAVE_CYCLES", 1)),
        "valu_util": d.get("SQ_INSTS_VALU", 0) * 2 / max(1.0, d.get("SQ_BUSY_CU_CYCLES", 1) * 16),
    }))
rows.sort(reverse=True)
out = {}
for _, k, m in rows[:14]:
    print(k[:60].ljust(60), " ".join(f"{a}={b:.3g}" for a, b in m.items()))
    out[k] = m
json.dump(out, open(os.path.join(ROOT, "gpurun_out", "issue", "summary.json"), "w"), indent=1)
