#!/bin/bash
# A/B/C: build/ab/libA.so, build/ab/libB1.so and libpcadv.so (the tree),
# alternated 3x in one call (tools/ab_feat.py: feature pair and step graph).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for i in 1 2 3; do
  PCADV_LIB=build/ab/libA.so timeout -k 10 120 python tools/ab_feat.py A 2>&1 | grep AB || exit 1
  PCADV_LIB=build/ab/libB1.so timeout -k 10 120 python tools/ab_feat.py B1 2>&1 | grep AB || exit 1
  timeout -k 10 120 python tools/ab_feat.py B 2>&1 | grep AB || exit 1
done
