#!/bin/bash
# Baseline check on a fresh box: the GPU suite, per-phase stamps of the
# feature forward / backward and the tail (diagnostic build), then the adv
# and cls benches.  Each GPU step has its own time limit; the first failure
# ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/b_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/b_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/fwd_stamps.py > gpurun_out/b_stamps.log 2>&1 || { echo "stamps failed"; tail -5 gpurun_out/b_stamps.log; exit 1; }
grep -v amdgpu.ids gpurun_out/b_stamps.log
timeout -k 10 120 python tools/tail_stamps.py > gpurun_out/b_tail.log 2>&1 || { echo "tail stamps failed"; tail -5 gpurun_out/b_tail.log; exit 1; }
grep -v amdgpu.ids gpurun_out/b_tail.log | head -60
timeout -k 10 200 python bench.py --steps 300 --warmup 30 --no-cpu > gpurun_out/b_bench.log 2>&1 || { echo "bench failed"; exit 1; }
grep metric gpurun_out/b_bench.log | cut -c1-300
timeout -k 10 200 python bench.py --config cls --steps 300 --warmup 30 --no-cpu > gpurun_out/b_cls.log 2>&1 || { echo "cls bench failed"; exit 1; }
grep metric gpurun_out/b_cls.log | cut -c1-300
