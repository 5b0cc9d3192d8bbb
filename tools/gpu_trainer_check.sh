#!/bin/bash
# The trainer fast path on the GPU: the data/trainer tests, then bench.py
# --config trainer (run_training end to end over DeviceCloudLoaders).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r03c}
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/${tag}_${name}.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -5 "gpurun_out/${tag}_${name}.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step pytest 600 python -u -m pytest tests/test_gpu_data.py -m gpu -v --timeout 180 --timeout-method thread -rf
step bench_trainer 600 python bench.py --config trainer --steps 300 --warmup 20
