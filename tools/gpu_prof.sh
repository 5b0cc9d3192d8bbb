#!/bin/bash
# Kernel-trace profile of the bench (no PMC counters in this pass).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-prof}
shift
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/$tag -o run --output-format csv -- python bench.py --no-cpu "$@" > gpurun_out/$tag.log 2>&1
rc=$?
echo "prof rc=$rc"; tail -3 gpurun_out/$tag.log
find gpurun_out/$tag -name "*stats*" | head
exit $rc
