#!/bin/bash
# A/B/...: every build/ab/lib*.so plus the tree's libpcadv.so ("tree"),
# alternated 3x in one call (tools/ab_feat.py: feature pair and step graph).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for i in 1 2 3; do
  for lib in build/ab/lib*.so; do
    tag=$(basename "$lib" .so); tag=${tag#lib}
    PCADV_LIB=$lib timeout -k 10 120 python tools/ab_feat.py "$tag" 2>&1 | grep AB || exit 1
  done
  timeout -k 10 120 python tools/ab_feat.py tree 2>&1 | grep AB || exit 1
done
