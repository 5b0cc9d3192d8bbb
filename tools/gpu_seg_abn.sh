#!/bin/bash
# Seg bench over every build/ab/lib*.so and the tree's library, alternated
# three times (one gpurun call: box-to-box variation is larger than the effects).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2 3; do
  for lib in build/ab/lib*.so adversarial_learning_on_pointclouds_amd/lib/libpcadv.so; do
    tag=$(basename "$lib" .so)
    PCADV_LIB=$lib timeout -k 10 200 python bench.py --config seg --steps 60 --warmup 10 --no-cpu > gpurun_out/sab_$tag$i.log 2>&1 || { echo "bench $tag failed"; tail -3 gpurun_out/sab_$tag$i.log; exit 1; }
    python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if '\"metric\"' in l][-1]); print('SAB $tag', d['ms_per_step'])" gpurun_out/sab_$tag$i.log
  done
done
