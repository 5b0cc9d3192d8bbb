#!/bin/bash
# GPU parity evidence: the whole -m gpu suite (verbose, per-test time limit),
# smoke() and a short bench.  Logs go to gpurun_out/<tag>_*.log; stops at the
# first step that crashes or times out.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r02}
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/${tag}_${name}.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -4 "gpurun_out/${tag}_${name}.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step pytest_gpu 1000 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread -rf
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 300 python bench.py --steps 50 --warmup 10 --cpu-seconds 5
