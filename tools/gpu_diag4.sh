#!/bin/bash
# Diagnostics: per-phase stamps (build/diag/libpcadv_stamps.so, copied there
# from `make stamps` for this run only) and a kernel trace of the adv bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r04d}
export PCADV_STAMPS_LIB=build/diag/libpcadv_stamps.so
timeout -k 10 120 python tools/fwd_stamps.py 64 1024 > gpurun_out/${tag}_stamps.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/${tag}_stamps.log | head -40
timeout -k 10 120 python tools/tail_stamps.py 32 1024 > gpurun_out/${tag}_tail_stamps.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/${tag}_tail_stamps.log | tail -32
unset PCADV_STAMPS_LIB
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_trace -o run --output-format csv -- python bench.py --no-cpu --steps 50 --warmup 10 > gpurun_out/${tag}_trace.log 2>&1 || exit $?
python tools/kstats.py gpurun_out/${tag}_trace/run_kernel_trace.csv 2>/dev/null | head -20
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_trace_seg -o run --output-format csv -- python bench.py --config seg --no-cpu --steps 5 --warmup 2 > gpurun_out/${tag}_trace_seg.log 2>&1 || exit $?
python tools/kstats.py gpurun_out/${tag}_trace_seg/run_kernel_trace.csv 2>/dev/null | head -24
