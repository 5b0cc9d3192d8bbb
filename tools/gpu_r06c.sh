#!/bin/bash
# Round 6 (second session): the data tests after the capturable-Adam step fix,
# then the fused feature-transform step's evidence and the cls trace
# (tools/gpu_r06b.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_data.py > gpurun_out/r06c_data_tests.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/r06c_data_tests.log | tail -8
if [ $rc -ne 0 ]; then tail -30 gpurun_out/r06c_data_tests.log; exit $rc; fi
bash tools/gpu_r06b.sh r06 || exit $?
