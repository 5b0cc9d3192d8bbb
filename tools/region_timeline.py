"""Whole-region timeline of a rocprofv3 kernel trace of `bench.py` (VERDICT r05
item 1): every graph replay (step) of every region, with the step's span
(its first kernel's start to the next step's first kernel's start), the idle
gap in front of it (previous kernel end -> its first kernel start) and the
sum of its kernels' durations; regions are split where the idle gap exceeds
--split us (the host synchronize between two timed regions).

    python tools/region_timeline.py run_kernel_trace.csv [--split 20] [--first K]
"""
import argparse
import csv

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--split", type=float, default=20.0)
ap.add_argument("--first", default="k_point_mlp", help="name of each step's first kernel")
args = ap.parse_args()

rows = list(csv.DictReader(open(args.trace)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ts = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
# a step = the kernels from one k_point_mlp up to the next one
starts = [i for i, t in enumerate(ts) if args.first in t[2]]
steps = []
for j, i0 in enumerate(starts):
    i1 = starts[j + 1] if j + 1 < len(starts) else len(ts)
    seg = ts[i0:i1]
    prev_end = max(t[1] for t in ts[:i0]) if i0 > 0 else seg[0][0]
    steps.append({"start": seg[0][0], "end": max(t[1] for t in seg), "n": len(seg),
                  "busy": sum(t[1] - t[0] for t in seg), "gap": seg[0][0] - prev_end,
                  "first_dur": seg[0][1] - seg[0][0]})
regions = [[]]
for s in steps:
    if regions[-1] and s["gap"] / 1e3 > args.split:
        regions.append([])
    regions[-1].append(s)
print("# rocprofv3 kernel-trace timestamps; one line per graph replay. span = this step's first "
      "kernel start -> next step's first kernel start (the last step: -> its last kernel end); "
      "gap = idle before the step's first kernel; busy = sum of its kernels' durations")
for ri, reg in enumerate(regions):
    t0 = reg[0]["start"]
    tot = reg[-1]["end"] - t0
    print(f"\n## region {ri}: {len(reg)} steps, first kernel -> last kernel end {tot / 1e3:.1f} us "
          f"({tot / 1e3 / len(reg):.2f} us/step); gap in front {reg[0]['gap'] / 1e3:.1f} us")
    for k, s in enumerate(reg):
        nxt = reg[k + 1]["start"] if k + 1 < len(reg) else s["end"]
        print(f"  step {k:3d} t={(s['start'] - t0) / 1e3:9.2f} span={(nxt - s['start']) / 1e3:7.2f} "
              f"gap={s['gap'] / 1e3:6.2f} busy={s['busy'] / 1e3:7.2f} kernels={s['n']:3d} "
              f"{args.first}={s['first_dur'] / 1e3:6.2f}")
