#!/bin/bash
# One lease: the FT / argmax-tie / T-Net / g13 / parity / distributed tests
# (no -x: every failure listed), the dp1 line with the unbucketed forms, and
# kernel traces of dp2 / dp2g.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_ft_step.py tests/test_gpu_argmax_ties.py tests/test_gpu_tnet.py tests/test_gpu_g13.py tests/test_gpu_parity.py tests/test_gpu_distributed.py > gpurun_out/r06b3_tests.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/r06b3_tests.log | tail -15
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 gpurun_out/r06b3_tests.log; exit $rc; fi
timeout -k 10 300 python bench.py --config dp1 --steps 200 --warmup 20 > gpurun_out/r06b3_dp1.log 2>&1
r=$?; echo "dp1 rc=$r"; grep -h '"metric"' gpurun_out/r06b3_dp1.log | cut -c1-900; [ $r -ne 0 ] && { tail -20 gpurun_out/r06b3_dp1.log; exit $r; }
for f in dp2 dp2g; do
  rm -rf gpurun_out/r06_dptrace_$f
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r06_dptrace_$f -o run --output-format csv -- python tools/dp_trace.py $f 30 > gpurun_out/r06_dptrace_$f.log 2>&1
  r=$?; echo "dptrace $f rc=$r"; [ $r -ne 0 ] && { tail -20 gpurun_out/r06_dptrace_$f.log; exit $r; }
done
exit $rc
