#!/bin/bash
# Phase stamps of the feature forward/backward, then the adv bench + trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python tools/fwd_stamps.py > gpurun_out/fs.log 2>&1
rc=$?; echo "stamps rc=$rc"; grep -A12 "k_feat_bwd_chunk" gpurun_out/fs.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_bench_trace.sh
