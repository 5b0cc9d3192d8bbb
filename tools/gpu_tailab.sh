#!/bin/bash
# Per-phase stamps of the feature backward's chunk launch inside the adv step
# (tools/tail_stamps.py) for each stamps library in build/diag/*_stamps.so
# (copied there for the run only), alternated twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  for lib in build/diag/*_stamps.so; do
    tag=$(basename "$lib" _stamps.so)
    PCADV_STAMPS_LIB=$lib timeout -k 10 120 python tools/tail_stamps.py 32 1024 > gpurun_out/tailab_${tag}_$i.log 2>&1 || exit $?
    echo "== $tag ($i)"; grep -v amdgpu.ids gpurun_out/tailab_${tag}_$i.log | grep -A40 "k_feat_bwd_chunk"
  done
done
