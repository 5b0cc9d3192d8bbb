"""One iteration's kernel timeline from a rocprofv3 kernel trace of
tools/dp_trace.py (the last complete iteration: from a k_point_mlp to the
next), with each kernel's queue, start, duration and the idle gap before it."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
st = [i for i, r in enumerate(rows) if "k_point_mlp" in r["Kernel_Name"]]
i0, i1 = st[-3], st[-2]
t0 = int(rows[i0]["Start_Timestamp"])
pe = t0
for r in rows[i0:i1]:
    s = (int(r["Start_Timestamp"]) - t0) / 1e3
    e = (int(r["End_Timestamp"]) - t0) / 1e3
    print(f"{s:8.2f} {e - s:7.2f} gap={s - (pe - t0) / 1e3:6.2f} q={r.get('Queue_Id', '?'):>2} "
          f"{r['Kernel_Name'].split('(')[0][:60]:60s} grid={r['Grid_Size_X']}")
    pe = max(pe, int(r["End_Timestamp"]))
print(f"iteration span {(int(rows[i1]['Start_Timestamp']) - t0) / 1e3:.2f} us")
