#!/bin/bash
# Kernel trace of the diagnostic (stamps) build's adversarial step, where each
# backward launch runs as a data-gradient launch and a weight-gradient launch:
# shows what the weight-gradient work adds to each dependent tail launch.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tail_split -o run -- python tools/tail_stamps.py > gpurun_out/tail_split.log 2>&1 || exit $?
python - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/tail_split/**/run_kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the last adversarial step's kernels: from the last k_point_mlp on
last = max(i for i, r in enumerate(rows) if "k_point_mlp" in r["Kernel_Name"])
t0 = int(rows[last]["Start_Timestamp"])
for r in rows[last:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1e3:8.2f} {(e - s) / 1e3:7.2f}  {r['Kernel_Name'][:60]}  grid={int(r['Grid_Size_X']) // int(r['Workgroup_Size_X'])}")
PY
