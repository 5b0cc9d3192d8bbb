#!/bin/bash
# Iteration loop on the GPU box: parity tests, then a kernel-trace profile of
# the bench.  Stops at the first crash/timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-iter}
timeout -k 10 900 python -m pytest tests -m gpu -q --timeout 300 -rf > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/$tag -o run --output-format csv -- python bench.py --no-cpu --steps 30 --warmup 5 > gpurun_out/$tag.log 2>&1
rc=$?; echo "prof rc=$rc"; grep '"metric"' gpurun_out/$tag.log | cut -c1-400
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu > gpurun_out/bench_$tag.log 2>&1
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_$tag.log | cut -c1-600
