"""Per-kernel (name + grid) means of the counters in rocprofv3 --pmc csv
directories: python tools/pmc_table.py DIR [DIR ...]."""
import collections
import csv
import glob
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            k = (row["Kernel_Name"].split("(")[0].replace("pcadv::", "")[-34:], row.get("Grid_Size", "?"))
            acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
for (name, grid), d in sorted(acc.items()):
    m = {c: sum(v) / len(v) for c, v in d.items()}
    extra = ""
    if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "GRBM_GUI_ACTIVE" in m and m["GRBM_GUI_ACTIVE"]:
        # MFMA busy per SIMD-cycle: busy cycles summed over SIMDs / (1024 SIMDs x GUI_ACTIVE / 8 XCDs)
        extra = f" mfma_util={m['SQ_VALU_MFMA_BUSY_CYCLES'] / (1024 * m['GRBM_GUI_ACTIVE'] / 8):.3f}"
    print(f"{name:34s} grid={grid:>9s} n={len(next(iter(d.values())))}{extra} " +
          " ".join(f"{c.replace('SQ_', '')}={v:.4g}" for c, v in sorted(m.items())))
