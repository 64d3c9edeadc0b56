"""Per-kernel stats (ms per frame) from a rocprofv3 rocpd SQLite database:
    python3 tools/rocpd_stats.py DB FRAMES [MIN_GRID_THREADS]
MIN_GRID_THREADS keeps only dispatches with at least that many threads (to
separate a large build's launches from small ones)."""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    frames = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    min_grid = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    where = f"where grid_x * grid_y * grid_z >= {min_grid}" if min_grid and "grid_x" in cols else ""
    rows = c.execute(f"select {name}, count(*), sum(end - start), avg(end - start) from kernels {where} "
                     f"group by {name} order by sum(end - start) desc").fetchall()
    tot = sum(r[2] for r in rows)
    for n, cnt, s, a in rows:
        print(f"{n.split('(')[0][:64]:64s} calls={cnt:5d} ms/frame={s / 1e6 / frames:8.3f} avg_us={a / 1e3:9.1f}")
    print(f"total kernel ms/frame {tot / 1e6 / frames:.2f}")


if __name__ == "__main__":
    main()
