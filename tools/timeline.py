#!/usr/bin/env python3
"""Per-queue timeline of the last bench frame from a rocprofv3 --kernel-trace
csv: 5-ms windows, busy ms and the top kernels of each queue, and per-phase
kernel overlap (which kernels ran beside which).
    python3 tools/timeline.py <..._kernel_trace.csv> [window_ms]
The last frame spans from the first launch after the previous frame's
k_resolve to its own k_resolve."""
import collections
import csv
import re
import sys


def short(name):
    n = re.sub(r"\(.*", "", name)
    n = n.replace("void ", "").replace("pmd::", "")
    return n[:48]


def main():
    path = sys.argv[1]
    win = float(sys.argv[2]) if len(sys.argv) > 2 else 5.0
    rows = list(csv.DictReader(open(path)))
    ks = []
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        ks.append((s, e, r.get("Queue_Id") or r.get("Stream_Id") or "?", short(r["Kernel_Name"])))
    ks.sort()
    # frames end with k_resolve; the last frame starts at the first launch
    # after the previous frame's k_resolve
    res = [k for k in ks if k[3].startswith("k_resolve")]
    if len(res) < 2:
        print("fewer than two frames (k_resolve launches) in the trace")
        return
    prev_end = res[-2][1]
    frame = [k for k in ks if k[0] >= prev_end and k[0] <= res[-1][1]]
    t0 = min(k[0] for k in frame)
    t1 = max(k[1] for k in frame)
    print(f"frame span {(t1 - t0) / 1e6:.1f} ms (first kernel start -> last kernel end); per HIP queue, "
          f"{win:g}-ms windows: busy ms, top kernels")
    byq = collections.defaultdict(list)
    for k in frame:
        byq[k[2]].append(k)
    for q in sorted(byq):
        print(f"\nqueue {q}")
        nwin = int((t1 - t0) / (win * 1e6)) + 1
        for w in range(nwin):
            a, b = t0 + w * win * 1e6, t0 + (w + 1) * win * 1e6
            per = collections.Counter()
            for s, e, _, n in byq[q]:
                ov = min(e, b) - max(s, a)
                if ov > 0:
                    per[n] += ov / 1e6
            busy = sum(per.values())
            if busy <= 0:
                continue
            top = ", ".join(f"{n} {v:.1f}" for n, v in per.most_common(3))
            print(f"  {w * win:6.0f}-{(w + 1) * win:<6.0f} ms  busy {min(busy, win):4.1f}  {top}")


if __name__ == "__main__":
    main()
