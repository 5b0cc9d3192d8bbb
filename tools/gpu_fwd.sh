#!/bin/bash
# Forward iteration: feature parity tests, stamps, kernel trace of the forward/backward driver.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -rf > gpurun_out/q_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/q_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python tools/fwd_stamps.py > gpurun_out/q_stamps.log 2>&1
rc=$?; echo "stamps rc=$rc"; grep -v amdgpu.ids gpurun_out/q_stamps.log | head -14
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/f_trace -o run --output-format csv -- python tools/feat_fwd_run.py 20 > gpurun_out/f_trace.log 2>&1
rc=$?; echo "trace rc=$rc"
python tools/kstats.py gpurun_out/f_trace/run_kernel_trace.csv | head -6
