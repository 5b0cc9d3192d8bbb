#!/bin/bash
# GPU parity suite, K1/K2/backward phase stamps, adv bench + kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -rf > gpurun_out/q_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/q_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/fwd_stamps.py > gpurun_out/fs.log 2>&1
rc=$?; echo "stamps rc=$rc"; grep -B1 -A13 "k_point_mlp:" gpurun_out/fs.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_bench_trace.sh
