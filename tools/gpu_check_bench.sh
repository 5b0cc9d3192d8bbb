#!/bin/bash
# Quick evidence call: SQ counters of the feature kernels, the new parity test
# of pcadv_conv4_max, and the adv / cls bench lines.  Stops at the first step
# that crashes or times out.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r03b}
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/${tag}_${name}.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -4 "gpurun_out/${tag}_${name}.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step pytest 300 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -rf -k "conv4_max_alone"
step bench 300 python bench.py --steps 50 --warmup 10 --cpu-seconds 6
step bench_cls 300 python bench.py --config cls --steps 50 --warmup 10 --no-cpu
bash tools/gpu_pmc_fwd.sh > "gpurun_out/${tag}_pmc.log" 2>&1; echo "pmc rc=$?"; tail -8 "gpurun_out/${tag}_pmc.log"
