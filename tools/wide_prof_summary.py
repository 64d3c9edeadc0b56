#!/usr/bin/env python3
"""Summary of tools/gpu_wide_prof.sh: profiles/<tag>_wide_kernel_stats.csv (the
rocprofv3 stats, copied) and profiles/<tag>_wide_pmc.json (per launch of each
gather kernel: HBM bytes as in tools/pmc_summary.py -- FETCH_SIZE doubled,
KiB -> B -- and the SQ wave counters).
    python3 tools/wide_prof_summary.py <tag> [gpurun_out/wide_prof/lib]"""
import glob
import json
import os
import shutil
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import pmc_table  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1]
src = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "gpurun_out", "wide_prof", "lib")
stats = glob.glob(os.path.join(src, "trace", "**", "*kernel_stats.csv"), recursive=True)
shutil.copy(stats[0], os.path.join(ROOT, "profiles", f"{tag}_wide_kernel_stats.csv"))
res = {}
for part in ("pmc_fetch", "pmc_write", "pmc_sq"):
    files = glob.glob(os.path.join(src, part, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        continue
    for k, v in pmc_table(files[0]).items():
        if "wide" not in k and "gather" not in k:
            continue
        res.setdefault(k, {}).update(v)
out = {}
for k, v in res.items():
    e = {c: v[c] for c in sorted(v) if c != "launches"}
    if "FETCH_SIZE" in v:
        e["hbm_read_bytes"] = 2 * v["FETCH_SIZE"] * 1024
    if "WRITE_SIZE" in v:
        e["hbm_write_bytes"] = v["WRITE_SIZE"] * 1024
    if "SQ_WAVE_CYCLES" in v and v.get("SQ_WAVE_CYCLES"):
        e["wait_frac"] = v.get("SQ_WAIT_ANY", 0) / v["SQ_WAVE_CYCLES"]
    out[k] = e
json.dump({"note": "per launch; FETCH_SIZE doubled (gfx950), KiB -> B", "kernels": out},
          open(os.path.join(ROOT, "profiles", f"{tag}_wide_pmc.json"), "w"), indent=1)
for k, e in out.items():
    print(k[:90], {c: round(x, 3) if isinstance(x, float) else x for c, x in e.items()
                   if c in ("hbm_read_bytes", "hbm_write_bytes", "wait_frac", "SQ_WAVES")})
