#!/bin/bash
# Round 6: where the cls step's hit sort runs.  A = ablib/libA.so built with
# -DPCADV_CLS_PRESORT=0 (the chunk workgroups sort their own hits), B = this
# tree (the sort rides in k_cls_head's idle workgroups).  cls bench alternated
# three times, then a kernel trace of A.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r06j}
for i in 1 2 3; do
  for v in A B; do
    if [ $v = A ]; then lib=ablib/libA.so; else lib=adversarial_learning_on_pointclouds_amd/lib/libpcadv.so; fi
    PCADV_LIB=$lib timeout -k 10 200 python bench.py --config cls --steps 300 --warmup 30 --no-cpu > gpurun_out/${tag}_$v$i.log 2>&1 || { echo "bench $v failed"; tail -20 gpurun_out/${tag}_$v$i.log; exit 1; }
    python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if '\"metric\"' in l][-1]); print('$v', d['ms_per_step'])" gpurun_out/${tag}_$v$i.log
  done
done
rm -rf gpurun_out/${tag}_trace
PCADV_LIB=ablib/libA.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_trace -o run --output-format csv -- python bench.py --config cls --no-cpu --steps 20 --warmup 5 > gpurun_out/${tag}_trace.log 2>&1 || { echo "trace rc=$?"; exit 1; }
echo trace ok
