#!/bin/bash
# The GPU suite, then the adv and cls benches alternated between
# build/ab/libA.so (A) and this tree's library (B), three times each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/ab_pytest.log
[ $rc -eq 0 ] || exit $rc
for cfg in adv cls; do
  for i in 1 2 3; do
    for v in A B; do
      if [ $v = A ]; then lib=build/ab/libA.so; else lib=adversarial_learning_on_pointclouds_amd/lib/libpcadv.so; fi
      PCADV_LIB=$lib timeout -k 10 200 python bench.py --config $cfg --steps 300 --warmup 30 --no-cpu > gpurun_out/ab_${cfg}_$v$i.log 2>&1 || { echo "bench $cfg $v failed"; exit 1; }
      python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if '\"metric\"' in l][-1]); print('$cfg $v', d['ms_per_step'])" gpurun_out/ab_${cfg}_$v$i.log
    done
  done
done
