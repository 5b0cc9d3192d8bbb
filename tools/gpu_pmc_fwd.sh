#!/bin/bash
# SQ counter passes over the feature forward/backward kernels (one pass each).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set -d gpurun_out/pmc$i -o run --output-format csv -- python tools/feat_fwd_run.py 3 > gpurun_out/pmc$i.log 2>&1
  rc=$?; echo "pmc$i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc$i.log; exit $rc; fi
done
python - <<'PY'
import csv, glob, collections
for i in (1, 2):
    f = glob.glob(f"gpurun_out/pmc{i}/**/*counter_collection.csv", recursive=True)[0]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"].split("(")[0][-28:]
        acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k, d in acc.items():
        print(k, {c: round(sum(v) / len(v)) for c, v in d.items()})
PY
