#!/bin/bash
# Seg: the GEMM-engine tests, then the seg bench alternated between build/ab/libA.so (A)
# and this tree's library (B), three times each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_seg.py -m gpu -q --timeout 600 --timeout-method thread -rf -x > gpurun_out/sab_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/sab_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
for i in 1 2 3; do
  for v in A B; do
    if [ $v = A ]; then lib=build/ab/libA.so; else lib=adversarial_learning_on_pointclouds_amd/lib/libpcadv.so; fi
    PCADV_LIB=$lib timeout -k 10 300 python bench.py --config seg --steps 30 --warmup 3 --no-cpu > gpurun_out/sab_$v$i.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/sab_$v$i.log; exit 1; }
    python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if '\"metric\"' in l][-1]); print('$v', d['ms_per_step'])" gpurun_out/sab_$v$i.log
  done
done
