#!/bin/bash
# One lease: the round-6 tests (fused feature-transform step, strict g13, DP),
# the dp1 / adv_ft bench lines, the adv_ft and cls profiles, and the argmax
# certification A/B.  A failing pytest (rc 1) does not stop the evidence steps;
# a time limit, abort or crash does.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_ft_step.py tests/test_gpu_g13.py tests/test_gpu_distributed.py -k "ft_step or g13 or semi_refused or rccl or dp_trainer" > gpurun_out/r06a_tests.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|PASSED|FAILED" gpurun_out/r06a_tests.log | tail -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 gpurun_out/r06a_tests.log; exit $rc; fi
for s in dp1 adv_ft adv_ft_body; do
  case $s in
    dp1) a="--config dp1 --steps 200 --warmup 20" ;;
    adv_ft) a="--config adv_ft --steps 100 --warmup 10 --no-cpu" ;;
    adv_ft_body) a="--config adv_ft --ft-body --steps 100 --warmup 10 --no-cpu" ;;
  esac
  timeout -k 10 300 python bench.py $a > gpurun_out/r06a_$s.log 2>&1
  r=$?; echo "$s rc=$r"; grep -h '"metric"' gpurun_out/r06a_$s.log | cut -c1-700
  if [ $r -ne 0 ]; then tail -30 gpurun_out/r06a_$s.log; exit $r; fi
done
bash tools/gpu_r06b.sh r06 || exit $?
bash tools/gpu_cert_ab.sh r06_cert || exit $?
exit $rc
