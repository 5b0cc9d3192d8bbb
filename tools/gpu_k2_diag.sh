#!/bin/bash
# k_conv4_max diagnostic variants (PCADV_C4_DIAG: 1 no screening, 2 no staging,
# 4 one-instruction keys) against the product library, alternated twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for i in 1 2; do
  for v in base D1 D2 D4; do
    if [ $v = base ]; then lib=adversarial_learning_on_pointclouds_amd/lib/libpcadv.so; else lib=build/ab/lib$v.so; fi
    out=$(PCADV_LIB=$lib timeout -k 10 120 python tools/k2_time.py 64 1024 fp32) || { echo "$v failed"; exit 1; }
    echo "$v fp32 $out"
    out=$(PCADV_LIB=$lib timeout -k 10 120 python tools/k2_time.py 32 1024 bf16) || { echo "$v failed"; exit 1; }
    echo "$v bf16 $out"
  done
done
