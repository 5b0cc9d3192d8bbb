#!/bin/bash
# Seg: the new GPU tests, then the seg bench with the weight-gradient finishes
# deferred (B) or one launch after each (A), alternated three times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_seg.py -x -q --timeout 300 --timeout-method thread > gpurun_out/sd_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/sd_pytest.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for v in 0 1; do
    PCADV_WGRAD_DEFER=$v timeout -k 10 200 python bench.py --config seg --steps 60 --warmup 10 --no-cpu > gpurun_out/sd_$v$i.log 2>&1 || { echo "bench $v failed"; tail -3 gpurun_out/sd_$v$i.log; exit 1; }
    python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if '\"metric\"' in l][-1]); print('defer=$v', d['ms_per_step'])" gpurun_out/sd_$v$i.log
  done
done
