#!/bin/bash
# seg path on the GPU box: parity tests, bench line, kernel trace summary
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_seg.py -x -q --timeout 120 --timeout-method thread > gpurun_out/seg_tests.log 2>&1
rc=$?; tail -3 gpurun_out/seg_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config seg --steps 20 --warmup 3 > gpurun_out/segb.log 2>&1 || exit $?
tail -1 gpurun_out/segb.log
rm -rf gpurun_out/seg_trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/seg_trace -o run --output-format csv -- python bench.py --config seg --steps 5 --warmup 1 --no-cpu > gpurun_out/seg_trace.log 2>&1 || exit $?
python tools/kstats.py gpurun_out/seg_trace/run_kernel_trace.csv > gpurun_out/seg_kstats.txt && head -40 gpurun_out/seg_kstats.txt
