#!/bin/bash
# The -m gpu suite only (verbose, per-test time limit); log to gpurun_out/<tag>_pytest_gpu.log
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r02}
shift
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -rf "$@" \
  > "gpurun_out/${tag}_pytest_gpu.log" 2>&1
rc=$?
echo "rc=$rc"; tail -40 "gpurun_out/${tag}_pytest_gpu.log"
exit $rc
