"""Per-kernel average durations from a rocprofv3 database (rocpd .db):
    python tools/trace_db_stats.py DIR_OR_DB [last_n_steps_kernels]
Groups dispatches by kernel name and grid; prints average/min durations."""
import glob
import os
import sqlite3
import sys
from collections import defaultdict


def main():
    p = sys.argv[1]
    f = p if p.endswith(".db") else glob.glob(os.path.join(p, "**", "*.db"), recursive=True)[0]
    c = sqlite3.connect(f)
    rows = c.execute("select name, grid_x, grid_y, workgroup_x, duration from kernels").fetchall()
    agg = defaultdict(list)
    for name, gx, gy, wx, d in rows:
        agg[(name[:60], gx // max(wx, 1), gy)].append(d)
    out = sorted(agg.items(), key=lambda kv: -sum(kv[1]))
    for (name, gx, gy), ds in out[:24]:
        ds.sort()
        print(f"{sum(ds) / len(ds) / 1e3:8.2f} us  med {ds[len(ds) // 2] / 1e3:8.2f}  x{len(ds):6d}  "
              f"grid {gx}x{gy}  {name}")


if __name__ == "__main__":
    main()
