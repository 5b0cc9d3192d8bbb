#!/bin/bash
# A/B of a build variant on the cls bench (configs[1], bf16 mode, 300 steps):
# A = ablib/libA.so, B = this tree's library, alternated three times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:?tag}
for i in 1 2 3; do
  for v in A B; do
    if [ $v = A ]; then lib=ablib/libA.so; else lib=adversarial_learning_on_pointclouds_amd/lib/libpcadv.so; fi
    PCADV_LIB=$lib timeout -k 10 200 python bench.py --config cls --steps 300 --warmup 30 --no-cpu > gpurun_out/${tag}_cls_$v$i.log 2>&1 || { echo "bench $v failed"; tail -20 gpurun_out/${tag}_cls_$v$i.log; exit 1; }
    python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if '\"metric\"' in l][-1]); r=d.get('roofline') or {}; print('$v cls', d['ms_per_step'], r.get('pair', {}).get('avg_us'))" gpurun_out/${tag}_cls_$v$i.log
  done
done
