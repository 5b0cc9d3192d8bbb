#!/bin/bash
# Adv bench (no CPU leg) + kernel trace summary: the quick perf loop.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu > gpurun_out/q_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep metric gpurun_out/q_bench.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/q_trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/q_trace -o run --output-format csv -- python bench.py --no-cpu --steps 30 --warmup 5 > gpurun_out/q_trace.log 2>&1
rc=$?; echo "trace rc=$rc"
python tools/kstats.py gpurun_out/q_trace/run_kernel_trace.csv > gpurun_out/q_kstats.txt; head -18 gpurun_out/q_kstats.txt
