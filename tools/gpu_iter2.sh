#!/bin/bash
# GPU parity suite, then the adv bench + kernel trace (the quick perf loop).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -rf > gpurun_out/q_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/q_pytest.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_bench_trace.sh
