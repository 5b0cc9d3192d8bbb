#!/bin/bash
# Quick iteration on the GPU box: parity tests, phase stamps, short bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -rf > gpurun_out/q_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/q_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python tools/fwd_stamps.py > gpurun_out/q_stamps.log 2>&1
rc=$?; echo "stamps rc=$rc"; cat gpurun_out/q_stamps.log | grep -v amdgpu.ids
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu > gpurun_out/q_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep metric gpurun_out/q_bench.log | cut -c1-330
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/q_trace -o run --output-format csv -- python bench.py --no-cpu --steps 30 --warmup 5 > gpurun_out/q_trace.log 2>&1
rc=$?; echo "trace rc=$rc"
python tools/kstats.py gpurun_out/q_trace/run_kernel_trace.csv | head -24
