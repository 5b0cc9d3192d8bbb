#!/bin/bash
# A/B of variant libraries in build/abx/ (copied there only for the run) against
# the tree's libpcadv.so: the feature-forward parity tests on each variant, then
# tools/ab_feat.py alternated 3x (feature pair + step graph).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in build/abx/lib*.so; do
  tag=$(basename "$lib" .so); tag=${tag#lib}
  PCADV_LIB=$lib timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 300 --timeout-method thread -k "feat or conv4 or argmax or adv_step" > gpurun_out/abx_$tag.log 2>&1
  rc=$?; echo "$tag tests rc=$rc: $(tail -1 gpurun_out/abx_$tag.log)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
for i in 1 2 3; do
  for lib in build/abx/lib*.so; do
    tag=$(basename "$lib" .so); tag=${tag#lib}
    PCADV_LIB=$lib timeout -k 10 120 python tools/ab_feat.py "$tag" 2>&1 | grep AB || exit 1
  done
  timeout -k 10 120 python tools/ab_feat.py tree 2>&1 | grep AB || exit 1
done
