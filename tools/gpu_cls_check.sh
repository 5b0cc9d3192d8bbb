#!/bin/bash
# The GPU suite, then the cls A/B (tools/gpu_cls_ab.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/c_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/c_pytest.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_cls_ab.sh
