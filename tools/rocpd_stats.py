"""Per-kernel totals from a rocprofv3 SQLite output (run_results.db):
python tools/rocpd_stats.py DB [--frames N] [--top K] [--csv OUT]."""
import argparse
import csv
import sqlite3


def kernel_stats(db):
    con = sqlite3.connect(db)
    cols = [r[1] for r in con.execute("pragma table_info(kernels)")]
    name = "name" if "name" in cols else "kernel_name"
    rows = con.execute(f"select {name}, count(*), sum(end - start), avg(end - start) from kernels "
                       f"group by {name} order by sum(end - start) desc").fetchall()
    return [(n, c, tot, avg) for n, c, tot, avg in rows]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--frames", type=float, default=1.0)
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--csv")
    a = ap.parse_args()
    rows = kernel_stats(a.db)
    total = sum(r[2] for r in rows)
    for n, c, tot, avg in rows[: a.top]:
        print(f"{n.split('(')[0][:58]:58s} calls={c:5d} ms/frame={tot / 1e6 / a.frames:8.2f} "
              f"avg_us={avg / 1e3:9.1f} {100 * tot / total:5.1f}%")
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
            for n, c, tot, avg in rows:
                w.writerow([n, c, tot, avg, 100 * tot / total])


if __name__ == "__main__":
    main()
