#!/bin/bash
# kernel trace of the cls bench (this tree's library)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03j_trace_cls -o run --output-format csv -- python bench.py --no-cpu --config cls --steps 50 --warmup 10 > gpurun_out/r03j.log 2>&1
