#!/bin/bash
# A/B of variant libraries in build/abx/ against the tree's on the trainer
# iteration (bench.py --config trainer: gather folded into k_point_mlp, the
# epilogue into the finishing launch): the trainer GPU tests on each variant,
# then alternated three times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
tree=adversarial_learning_on_pointclouds_amd/lib/libpcadv.so
for lib in build/abx/lib*.so; do
  tag=$(basename "$lib" .so)
  PCADV_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_data.py -m gpu -q -x --timeout 200 --timeout-method thread -k "trainer or fold or graphed" > gpurun_out/trab_$tag.log 2>&1
  rc=$?; echo "$tag tests rc=$rc: $(tail -1 gpurun_out/trab_$tag.log)"
  [ $rc -eq 0 ] || exit $rc
done
for i in 1 2 3; do
  for lib in build/abx/lib*.so $tree; do
    tag=$(basename "$lib" .so)
    PCADV_LIB=$lib timeout -k 10 200 python bench.py --config trainer --steps 300 --warmup 20 --no-cpu > gpurun_out/trab.log 2>&1 || exit 1
    python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/trab.log') if '\"metric\"' in l][-1]); print('AB', sys.argv[1], d['ms_per_step'])" "$tag"
  done
done
