#!/bin/bash
# One lease: FT / distributed / g13 tests after the deferred weight-gradient
# reductions, dx_relu and the one-graph DP default; the dp1 overhead line;
# then the adv_ft evidence (trace, PMC traffic, MFMA busy, bench line) and
# the cls trace via tools/gpu_r06b.sh.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v -s --timeout 200 --timeout-method thread tests/test_gpu_ft_step.py tests/test_gpu_distributed.py tests/test_gpu_g13.py tests/test_gpu_tnet.py > gpurun_out/r06b4_tests.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/r06b4_tests.log | tail -15
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 gpurun_out/r06b4_tests.log; exit $rc; fi
timeout -k 10 300 python bench.py --config dp1 --steps 200 --warmup 20 > gpurun_out/r06b4_dp1.log 2>&1
r=$?; echo "dp1 rc=$r"; grep -h '"metric"' gpurun_out/r06b4_dp1.log | cut -c1-900; [ $r -ne 0 ] && { tail -20 gpurun_out/r06b4_dp1.log; exit $r; }
bash tools/gpu_r06b.sh r06 || exit $?
exit $rc
