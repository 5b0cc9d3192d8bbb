#!/bin/bash
# Seg: the seg GPU tests, then the seg bench with environment A ("$1", e.g.
# PCADV_GEMM_PAIR=0) against B ("$2", may be empty), alternated three times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_seg.py -x -q --timeout 300 --timeout-method thread > gpurun_out/se_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/se_pytest.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for v in A B; do
    if [ $v = A ]; then e="$1"; else e="$2"; fi
    env $e timeout -k 10 200 python bench.py --config seg --steps 60 --warmup 10 --no-cpu > gpurun_out/se_$v$i.log 2>&1 || { echo "bench $v failed"; tail -3 gpurun_out/se_$v$i.log; exit 1; }
    python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if '\"metric\"' in l][-1]); print('$v [$e]', d['ms_per_step'])" gpurun_out/se_$v$i.log
  done
done
