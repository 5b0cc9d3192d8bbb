#!/bin/bash
# Cls bench (configs[1], bf16 mode) alternated between build/ab/libA.so (A) and
# this tree's library (B), three times each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2 3; do
  for v in A B; do
    if [ $v = A ]; then lib=build/ab/libA.so; else lib=adversarial_learning_on_pointclouds_amd/lib/libpcadv.so; fi
    PCADV_LIB=$lib timeout -k 10 200 python bench.py --config cls --steps 300 --warmup 30 --no-cpu > gpurun_out/cab_$v$i.log 2>&1 || { echo "bench $v failed"; exit 1; }
    python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if '\"metric\"' in l][-1]); print('$v', d['ms_per_step'], d.get('roofline', {}).get('avg_launch_us'), d.get('roofline', {}).get('pair', {}).get('avg_us'))" gpurun_out/cab_$v$i.log
  done
done
