#!/bin/bash
# Round 6: the fused feature-transform step, the strict g13 checks, the DP
# overhead bench (one-rank RCCL) - tests first, then the bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r06a}
set -o pipefail
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/${tag}_${name}.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; grep -h -E '"metric"|passed|failed|Error' "gpurun_out/${tag}_${name}.log" | cut -c1-600 | tail -12
  if [ $rc -ne 0 ]; then tail -40 "gpurun_out/${tag}_${name}.log"; exit $rc; fi
}
step tests 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_ft_step.py tests/test_gpu_g13.py tests/test_gpu_distributed.py -k "ft_step or g13 or semi_refused or rccl or dp_trainer"
step dp1 300 python bench.py --config dp1 --steps 200 --warmup 20
step adv_ft 300 python bench.py --config adv_ft --steps 100 --warmup 10 --no-cpu
step adv_ft_body 300 python bench.py --config adv_ft --ft-body --steps 100 --warmup 10 --no-cpu
