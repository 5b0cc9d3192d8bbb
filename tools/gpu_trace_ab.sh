#!/bin/bash
# Kernel-trace medians of the adv and cls benches for each library in
# build/abx/ and the tree's (PCADV_LIB): per-kernel A/B where the step time is
# too noisy to separate a sub-microsecond change.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
tree=adversarial_learning_on_pointclouds_amd/lib/libpcadv.so
for cfg in adv cls; do
  for lib in build/abx/lib*.so $tree; do
    tag=$(basename "$lib" .so); tag=${tag#lib}_$cfg
    rm -rf gpurun_out/tab_$tag
    PCADV_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/tab_$tag -o run --output-format csv -- python bench.py --config $cfg --no-cpu --steps 100 --warmup 10 --repeats 1 > gpurun_out/tab_$tag.log 2>&1
    rc=$?; echo "$tag rc=$rc"
    [ $rc -eq 0 ] || exit $rc
    python tools/kstats.py gpurun_out/tab_$tag/run_kernel_trace.csv > gpurun_out/tab_$tag.txt
  done
done
for f in gpurun_out/tab_*.txt; do echo "== $f"; grep -v rocclr "$f" | head -16; done
