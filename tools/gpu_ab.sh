#!/bin/bash
# A/B: libpcadv.so (B, the tree) vs build/ab/libA.so (A), alternated 3x.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for i in 1 2 3; do
  PCADV_LIB=build/ab/libA.so timeout -k 10 120 python tools/ab_feat.py A 2>&1 | grep AB || exit 1
  timeout -k 10 120 python tools/ab_feat.py B 2>&1 | grep AB || exit 1
done
