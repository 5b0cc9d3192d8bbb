#!/bin/bash
# A/B of the diagnostic stamps build: build/stamps (A) vs build/stampsB (B),
# alternated twice on one box; prints the feature-backward summaries.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for v in A B; do
    lib=build/stamps/libpcadv_stamps.so; [ $v = B ] && lib=build/stampsB/libpcadv_stamps.so
    PCADV_STAMPS_LIB=$lib timeout -k 10 120 python -u tools/fwd_stamps.py > gpurun_out/ab_${v}${r}.log 2>&1 || exit $?
    echo "== $v run $r"; grep -E "kernel end|batch1 (a|b|gather)|event time" gpurun_out/ab_${v}${r}.log | grep -v k_conv4 | tail -6
  done
done
