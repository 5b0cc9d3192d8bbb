"""Print one step's kernel timeline from a rocprofv3 kernel trace (the last
complete graph replay: a k_point_mlp followed by the step's kernels)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "k_point_mlp" in r["Kernel_Name"]
          and i + 2 < len(rows) and "k_linear_fwd" in rows[i + 2]["Kernel_Name"]]
which = int(sys.argv[2]) if len(sys.argv) > 2 else -2
i0 = starts[which]
i1 = starts[which + 1] if which + 1 < len(starts) else len(rows)
t0 = int(rows[i0]["Start_Timestamp"])
print("# rocprofv3 kernel-trace timestamps (us from the step's first kernel). Gaps of about +-1 us "
      "(negative ones included) are skew between dispatch records, not idle time; the step time "
      "is bench.py's event timing.")
prev_end = t0
for r in rows[i0:i1]:
    s = (int(r["Start_Timestamp"]) - t0) / 1e3
    e = (int(r["End_Timestamp"]) - t0) / 1e3
    gap = s - (prev_end - t0) / 1e3
    prev_end = max(prev_end, int(r["End_Timestamp"]))
    name = r["Kernel_Name"].split("(")[0].replace("pcadv::", "")
    print(f"{s:8.2f} {e:8.2f} dur={e - s:6.2f} gap={gap:6.2f} q={r.get('Queue_Id', '?'):>2} "
          f"{name:22s} grid={r['Grid_Size_X']}")
print(f"step span: {(int(rows[i1]['Start_Timestamp']) - t0) / 1e3 if i1 < len(rows) else float('nan'):.2f} us")
