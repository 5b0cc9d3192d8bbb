"""MFMA utilisation per kernel from a rocprofv3 --pmc pass that collected
SQ_VALU_MFMA_BUSY_CYCLES and GRBM_GUI_ACTIVE (plus --kernel-trace in the same
run, for the dispatch durations).

    python tools/pmc_mfma.py <pmc_dir> <out.json> <label> [kernel-prefix ...]

SQ_VALU_MFMA_BUSY_CYCLES is summed over the chip's 1024 SIMDs and counts
matrix-pipe cycles (32 per v_mfma_f32_32x32x16_bf16, MI355X_MICROARCH.md).
GRBM_GUI_ACTIVE is the dispatch's GPU-busy cycles summed over the 8 XCDs, so

    mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 x GRBM_GUI_ACTIVE / 8)

is the fraction of SIMD-cycles the matrix pipe was busy during the dispatch
(GUI_ACTIVE includes the dispatch's ramp-up and drain, so this is a lower
bound for short launches).  clock_ghz = GRBM_GUI_ACTIVE / 8 / the profiled
dispatch's kernel-trace duration; mfma_busy_at_2p4ghz prices the busy cycles
against that duration at the nominal 2.4 GHz instead.
"""
import collections
import csv
import glob
import json
import os
import statistics
import sys

SIMDS = 1024


def _rows(d, pattern):
    fs = glob.glob(os.path.join(d, "**", pattern), recursive=True)
    return list(csv.DictReader(open(fs[0]))) if fs else []


def main():
    d, out, label = sys.argv[1], sys.argv[2], sys.argv[3]
    prefixes = sys.argv[4:]
    per = collections.defaultdict(lambda: collections.defaultdict(dict))
    names = {}
    for r in _rows(d, "*counter_collection.csv"):
        kid = r.get("Dispatch_Id") or r.get("Correlation_Id")
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("pcadv::", "")
        key = (name, r.get("Grid_Size", "?"))
        names[kid] = key
        per[key][kid][r["Counter_Name"]] = per[key][kid].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    dur = {}
    for r in _rows(d, "*kernel_trace.csv"):
        kid = r.get("Dispatch_Id") or r.get("Correlation_Id")
        dur[kid] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    res = {}
    for key, disp in per.items():
        name, grid = key
        if prefixes and not any(name.startswith(p) for p in prefixes):
            continue
        busy = [c.get("SQ_VALU_MFMA_BUSY_CYCLES") for c in disp.values()]
        gui = [c.get("GRBM_GUI_ACTIVE") for c in disp.values()]
        if None in busy or None in gui:
            continue
        util = [b / (SIMDS * g / 8) for b, g in zip(busy, gui) if g]
        ent = {"launches": len(disp),
               "SQ_VALU_MFMA_BUSY_CYCLES": statistics.median(busy),
               "GRBM_GUI_ACTIVE": statistics.median(gui),
               "mfma_busy": round(statistics.median(util), 4)}
        for c in ("SQ_BUSY_CYCLES", "SQ_INSTS_MFMA", "SQ_INSTS_VALU", "SQ_WAVES", "SQ_WAVE_CYCLES"):
            v = [x.get(c) for x in disp.values()]
            if None not in v:
                ent[c] = statistics.median(v)
        ds = [dur[k] for k in disp if k in dur]
        if ds:
            t = statistics.median(ds)
            ent["profiled_duration_us"] = round(t * 1e6, 2)
            ent["clock_ghz"] = round(ent["GRBM_GUI_ACTIVE"] / 8 / t / 1e9, 3)
            # the same busy cycles against the profiled duration at the nominal 2.4 GHz
            ent["mfma_busy_at_2p4ghz"] = round(ent["SQ_VALU_MFMA_BUSY_CYCLES"] / (SIMDS * t * 2.4e9), 4)
        res[f"{name} grid={grid}"] = ent
    for k, v in sorted(res.items(), key=lambda kv: -kv[1]["SQ_VALU_MFMA_BUSY_CYCLES"]):
        print(f"{k[:60]:60s} n={v['launches']:4d} mfma_busy={v['mfma_busy']:.3f} "
              f"dur={v.get('profiled_duration_us', 0):8.2f}us clk={v.get('clock_ghz', 0):.2f}")
    json.dump({"source": f"rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE ... "
                         f"of `{label}`",
               "definition": "mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs), "
                             "median over the profiled dispatches",
               "kernels": res}, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
