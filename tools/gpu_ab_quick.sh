#!/bin/bash
# A/B of a build variant: the adv bench (configs[2], 200 steps) and the
# run_training bench alternated three times between A = ablib/libA.so and
# B = this tree's library (--no-cpu).  Usage: bash tools/gpu_ab_quick.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:?tag}
for i in 1 2 3; do
  for v in A B; do
    if [ $v = A ]; then lib=ablib/libA.so; else lib=adversarial_learning_on_pointclouds_amd/lib/libpcadv.so; fi
    PCADV_LIB=$lib timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu > gpurun_out/${tag}_adv_$v$i.log 2>&1 || { echo "bench $v failed"; tail -20 gpurun_out/${tag}_adv_$v$i.log; exit 1; }
    PCADV_LIB=$lib timeout -k 10 200 python bench.py --config trainer --steps 300 --warmup 20 > gpurun_out/${tag}_tr_$v$i.log 2>&1 || { echo "trainer $v failed"; tail -20 gpurun_out/${tag}_tr_$v$i.log; exit 1; }
    python -c "
import json,sys
def ln(f):
    d=json.loads([l for l in open(f) if '\"metric\"' in l][-1]); return d['ms_per_step'], (d.get('roofline') or {}).get('pair', {}).get('avg_us')
print('$v adv', *ln(sys.argv[1]), 'trainer', ln(sys.argv[2])[0])" gpurun_out/${tag}_adv_$v$i.log gpurun_out/${tag}_tr_$v$i.log
  done
done
