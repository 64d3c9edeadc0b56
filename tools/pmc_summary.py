#!/usr/bin/env python3
"""Summarise a profiles_run.sh output directory into profiles/<tag>_*.

Writes:
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (copied)
  profiles/<tag>_pmc.json           per-kernel PMC totals per launch
  profiles/pmc_gather_global.json   HBM traffic of the dominant kernel (read by bench.py only
                                    while libpm_hip.so still has the profiled sha256)
HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are KiB;
gfx950 FETCH_SIZE reports 1/2 of a wide coalesced stream's bytes, so it is
doubled (uncalibrated for other access widths: noted in the JSON).
"""
import collections
import csv
import json
import os
import re
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import source_digest  # noqa: E402  (the identity bench.py checks)


def pmc_table(path):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    launches = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        per[k][r["Counter_Name"]] += float(r["Counter_Value"])
        launches[k].add(r["Dispatch_Id"])
    return {k: {c: v / max(1, len(launches[k])) for c, v in d.items()} | {"launches": len(launches[k])}
            for k, d in per.items()}


def main(tag="r01", src=os.path.join(ROOT, "gpurun_out", "prof"), workload=None):
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", f"{tag}_kernel_stats.csv"), os.path.join(dst, f"{tag}_kernel_stats.csv"))
    merged = collections.defaultdict(dict)
    for sub in ("pmc_fetch", "pmc_write", "pmc_sq"):
        p = os.path.join(src, sub, f"{tag}_counter_collection.csv")
        if os.path.exists(p):
            for k, d in pmc_table(p).items():
                merged[k].update(d)
    out = {}
    for k, d in merged.items():
        if d.get("FETCH_SIZE", 0) + d.get("WRITE_SIZE", 0) < 1 and "SQ_WAVES" not in d:
            continue
        e = dict(d)
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            e["hbm_bytes_per_launch"] = (2 * d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024
        out[k] = e
    with open(os.path.join(dst, f"{tag}_pmc.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    # the global-map gather phase: k_gather<1,...> (modes 0-11, 14) or the seeded pair
    # k_gather_level<1,...> launches (modes 12/13, default): per-phase sums
    g = [k for k in out if re.search(r"k_gather(_lead|_seeded|_level)?<1,", k)]
    sha_file = os.path.join(src, "lib.sha256")
    lib_sha = open(sha_file).read().split()[0] if os.path.exists(sha_file) else None
    if g and workload is not None:
        tot = lambda c: sum(out[k].get(c) or 0.0 for k in g) if all(c in out[k] for k in g) else None
        fetch, write = tot("FETCH_SIZE"), tot("WRITE_SIZE")
        with open(os.path.join(dst, "pmc_gather_global.json"), "w") as f:
            json.dump({"kernel": " + ".join(sorted(g)), "workload": workload, "tag": tag, "lib_sha256": lib_sha,
                       "src_sha256": source_digest(),
                       "fetch_kib": fetch, "write_kib": write,
                       "hbm_bytes_per_launch": (2 * fetch + write) * 1024 if fetch is not None and write is not None
                       else None,
                       "note": "per global-gather phase (sum of its kernels, one launch each per frame); "
                               "FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM (calibrated for wide coalesced "
                               "reads; this kernel gathers 16-B nodes, so the absolute is uncalibrated)"}, f,
                      indent=1)
    print(json.dumps({k[:60]: v.get("hbm_bytes_per_launch") for k, v in out.items()}, indent=1))


if __name__ == "__main__":
    tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
    main(tag, workload=["sponza", 10_000_000, 1_000_000, 1920, 1080, 1])
