#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for d in 0 1 2 3; do
  lib=build/stamps/libpcadv_d$d.so; [ $d = 0 ] && lib=build/stamps/libpcadv_stamps.so
  echo "=== diag $d"
  PCADV_STAMPS_LIB=$lib timeout -k 10 120 python tools/fwd_stamps.py 2>&1 | grep -A3 "k_conv4_max" | head -4
  rc=$?; [ $rc -ne 0 ] && exit $rc
done
