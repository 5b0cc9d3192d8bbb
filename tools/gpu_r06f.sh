#!/bin/bash
# Round 6: fork/join cost inside a replayed graph (tools/fork_join_probe.py)
# and the per-phase stamps of the feature forward / backward on the current
# kernels (diagnostic library, tools/fwd_stamps.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for d in 2 4 8; do
  timeout -k 10 120 python tools/fork_join_probe.py $d >> gpurun_out/r06f_fork_join.jsonl 2> gpurun_out/r06f_fork_join_$d.err || { echo "probe rc=$?"; tail gpurun_out/r06f_fork_join_$d.err; exit 1; }
done
cat gpurun_out/r06f_fork_join.jsonl
PCADV_STAMPS_LIB=stamps_tmp/libpcadv_stamps.so timeout -k 10 180 python -u tools/fwd_stamps.py > gpurun_out/r06f_feat_stamps.txt 2>&1 || { echo "stamps rc=$?"; tail -20 gpurun_out/r06f_feat_stamps.txt; exit 1; }
head -20 gpurun_out/r06f_feat_stamps.txt
