#!/bin/bash
# Seg: the seg GPU tests, then the seg bench under each environment setting
# given as an argument ("" = defaults), alternated three times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_seg.py -x -q --timeout 300 --timeout-method thread > gpurun_out/sc_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/sc_pytest.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  j=0
  for e in "$@"; do
    j=$((j+1))
    env $e timeout -k 10 200 python bench.py --config seg --steps 60 --warmup 10 --no-cpu > gpurun_out/sc_$j$i.log 2>&1 || { echo "bench [$e] failed"; tail -3 gpurun_out/sc_$j$i.log; exit 1; }
    python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if '\"metric\"' in l][-1]); print('[$e]', d['ms_per_step'])" gpurun_out/sc_$j$i.log
  done
done
