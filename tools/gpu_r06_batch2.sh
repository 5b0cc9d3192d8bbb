#!/bin/bash
# One lease: FT / T-Net / parity tests after the k_conv4_max ReLU epilogue and
# pcadv_concat2, the adv_ft line, and kernel traces of the three DP forms.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_ft_step.py tests/test_gpu_tnet.py tests/test_gpu_g13.py tests/test_gpu_parity.py > gpurun_out/r06b2_tests.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/r06b2_tests.log | tail -15
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 gpurun_out/r06b2_tests.log; exit $rc; fi
timeout -k 10 300 python bench.py --config adv_ft --steps 100 --warmup 10 --no-cpu > gpurun_out/r06b2_adv_ft.log 2>&1
r=$?; echo "adv_ft rc=$r"; grep -h '"metric"' gpurun_out/r06b2_adv_ft.log | cut -c1-400; [ $r -ne 0 ] && exit $r
for f in plain dp4 dp1g; do
  rm -rf gpurun_out/r06_dptrace_$f
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r06_dptrace_$f -o run --output-format csv -- python tools/dp_trace.py $f 30 > gpurun_out/r06_dptrace_$f.log 2>&1
  r=$?; echo "dptrace $f rc=$r"; [ $r -ne 0 ] && { tail -20 gpurun_out/r06_dptrace_$f.log; exit $r; }
done
exit $rc
