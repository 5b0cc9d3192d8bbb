#!/bin/bash
# Kernel-trace stats of the adversarial step graph for two libraries
# (build/ab/libA.so and the tree's libpcadv.so): per-kernel average durations.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PCADV_LIB=build/ab/libA.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/trA -o run -- python tools/ab_feat.py A > gpurun_out/trA.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/trB -o run -- python tools/ab_feat.py B > gpurun_out/trB.log 2>&1 || exit 1
for t in trA trB; do
  echo "== $t"; grep AB gpurun_out/$t.log
  python tools/trace_db_stats.py gpurun_out/$t | head -16
done
