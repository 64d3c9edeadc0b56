"""Per-frame kernel table from a rocprofv3 --stats kernel_stats.csv: python3 tools/kstats.py <csv> <frames> [top]."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
frames = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
top = int(sys.argv[3]) if len(sys.argv) > 3 else 16
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:top]:
    print(f"{float(r['TotalDurationNs']) / 1e6 / frames:9.2f} ms/frame  calls {int(r['Calls']) / frames:6.1f}  "
          f"avg {float(r['AverageNs']) / 1e6:8.3f}  {r['Name'][:80]}")
