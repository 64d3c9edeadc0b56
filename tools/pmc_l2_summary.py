#!/usr/bin/env python3
"""Summary of tools/pmc_l2.sh: per library, the gather kernels' L1->L2 read
requests, L1 accesses and L2 hit rate per launch.
    python3 tools/pmc_l2_summary.py [gpurun_out/pmc_l2]"""
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import pmc_table  # noqa: E402

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_l2"
for d in sorted(glob.glob(os.path.join(root, "*"))):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        continue
    t = pmc_table(files[0])
    print(f"== {os.path.basename(d)}")
    for k, v in sorted(t.items(), key=lambda kv: -kv[1].get("TCP_TCC_READ_REQ_sum", 0)):
        if "gather" not in k and "kd_" not in k and "ph_trace" not in k:
            continue
        h, m = v.get("TCC_HIT_sum", 0), v.get("TCC_MISS_sum", 0)
        print(f"  {k[:70]:70s} L1 acc {v.get('TCP_TOTAL_CACHE_ACCESSES_sum', 0) / 1e6:9.1f} M  "
              f"L2 req {v.get('TCP_TCC_READ_REQ_sum', 0) / 1e6:9.1f} M  L2 hit {h / max(1, h + m):.3f}  "
              f"miss {m / 1e6:8.1f} M")
