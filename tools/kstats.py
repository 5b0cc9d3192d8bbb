"""Summarise a rocprofv3 kernel trace: per kernel (and grid) average duration,
plus per-step accounting over the timed graph replays."""
import collections
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import kname  # noqa: E402

path = sys.argv[1]
rows = list(csv.DictReader(open(path)))
d = collections.defaultdict(list)
for x in rows:
    name = kname(x["Kernel_Name"])[:40]
    key = (name, x["Grid_Size_X"], x["Grid_Size_Y"], x["Workgroup_Size_X"])
    d[key].append((int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e3)
tot = 0
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    s = sorted(v)
    med = s[len(s) // 2]
    print(f"{k[0]:40s} grid={k[1]:>7s}x{k[2]:>3s} wg={k[3]:>4s} n={len(v):4d} med_us={med:8.2f} sum_ms={sum(v)/1e3:7.2f}")
