"""Per-kernel HBM traffic from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

    python tools/pmc_traffic.py <fetch_dir> <write_dir> [out.json]

rocprofv3 reports both derived counters in KiB per dispatch.  On gfx950
FETCH_SIZE counts half the bytes of wide coalesced reads (MI355X_MICROARCH.md,
HBM section: 128-B requests tallied at 64 B), so reads are doubled; WRITE_SIZE
is taken as is.  Both derive from the L2's memory-side requests, so
Infinity-Cache (MALL) hits are included: this is L2-miss traffic, an upper
bound on HBM bytes.  The two passes ran the same command, so dispatches are
matched by kernel name and averaged per launch.
"""
import collections
import csv
import glob
import json
import os
import re
import sys


def kname(raw):
    """Kernel name without arguments; mangled names rocprofv3 could not demangle
    (e.g. __bf16 parameters) are reduced to ns::name."""
    m = re.match(r"_ZN(\d+)(\w+)", raw)
    if m:
        n = int(m.group(1))
        ns, rest = m.group(2)[:n], m.group(2)[n:]
        m2 = re.match(r"(\d+)(\w+)", rest)
        if m2:
            return ns + "::" + m2.group(2)[:int(m2.group(1))]
    return raw.split("(")[0].replace("void ", "")


def load(d, counter):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    per = collections.defaultdict(list)
    for row in csv.DictReader(open(f)):
        if row["Counter_Name"] != counter:
            continue
        name = kname(row["Kernel_Name"])
        per[name].append(float(row["Counter_Value"]) * 1024.0)
    return per


def main():
    fetch = load(sys.argv[1], "FETCH_SIZE")
    write = load(sys.argv[2], "WRITE_SIZE")
    out = {}
    for name in sorted(set(fetch) | set(write)):
        fr, wr = fetch.get(name, []), write.get(name, [])
        if not fr or not wr:
            continue
        rd = 2.0 * sum(fr) / len(fr)
        wb = sum(wr) / len(wr)
        out[name] = {"launches": len(fr), "read_bytes": rd, "write_bytes": wb,
                     "traffic_bytes": rd + wb}
    for name, v in sorted(out.items(), key=lambda kv: -kv[1]["traffic_bytes"]):
        print(f"{name[:44]:44s} n={v['launches']:4d} read={v['read_bytes'] / 1e6:9.3f} MB "
              f"write={v['write_bytes'] / 1e6:9.3f} MB")
    if len(sys.argv) > 3:
        json.dump({"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE passes of "
                             "`python bench.py --no-cpu --steps 3 --warmup 1`; reads x2 "
                             "(gfx950 FETCH_SIZE halving), KiB -> bytes",
                   "kernels": out}, open(sys.argv[3], "w"), indent=1)


if __name__ == "__main__":
    main()
