#!/bin/bash
# Targeted GPU run of the tests a change touched (pytest -k expression), then
# smoke().  Logs under gpurun_out/<tag>_*.log; stops at a crash or time-out.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r03a}
expr=${2:-}
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/${tag}_${name}.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -6 "gpurun_out/${tag}_${name}.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
if [ -n "$expr" ]; then
  step pytest 1100 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread -rf -k "$expr"
else
  step pytest 1100 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread -rf
fi
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
