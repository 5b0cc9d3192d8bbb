#!/bin/bash
# A/B of variant libraries in build/abx/ (copied there only for the run) against
# the tree's libpcadv.so: the feature-forward parity tests on each library, then
# alternated 3x: tools/ab_feat.py (adv feature pair + step graph) or, with
# argument "cls", the configs[1] bench (bf16 cls step).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
mode=${1:-adv}
tree=adversarial_learning_on_pointclouds_amd/lib/libpcadv.so
for lib in build/abx/lib*.so $tree; do
  tag=$(basename "$lib" .so); tag=${tag#lib}
  PCADV_LIB=$lib timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 300 --timeout-method thread -k "feat or conv4 or argmax or adv_step or cls" > gpurun_out/abx_$tag.log 2>&1
  rc=$?; echo "$tag tests rc=$rc: $(tail -1 gpurun_out/abx_$tag.log)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
for i in 1 2 3; do
  for lib in build/abx/lib*.so $tree; do
    tag=$(basename "$lib" .so); tag=${tag#lib}
    if [ "$mode" = cls ]; then
      PCADV_LIB=$lib timeout -k 10 200 python bench.py --config cls --steps 300 --warmup 30 --no-cpu > gpurun_out/abx_cls_$tag.log 2>&1 || { echo "bench $tag failed"; exit 1; }
      python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if '\"metric\"' in l][-1]); r=d.get('roofline', {}); print('AB $tag', d['ms_per_step'], r.get('avg_launch_us'), r.get('pair', {}).get('avg_us'))" gpurun_out/abx_cls_$tag.log
    else
      PCADV_LIB=$lib timeout -k 10 120 python tools/ab_feat.py "$tag" 2>&1 | grep AB || exit 1
    fi
  done
done
