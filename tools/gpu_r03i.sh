#!/bin/bash
# k_cls_head: the cls GPU tests, smoke, then the cls bench A/B (build/ab/libA.so = before).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -k "cls or Cls or trainer" --timeout 300 --timeout-method thread -rf -x > gpurun_out/r03i_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r03i_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_cls_ab.sh
timeout -k 10 120 build/sync_bench > gpurun_out/sync_bench.log 2>&1 || { cat gpurun_out/sync_bench.log; exit 1; }
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 120 build/sync_bench > gpurun_out/sync_bench_pc0.log 2>&1 || { cat gpurun_out/sync_bench_pc0.log; exit 1; }
cat gpurun_out/sync_bench.log gpurun_out/sync_bench_pc0.log
