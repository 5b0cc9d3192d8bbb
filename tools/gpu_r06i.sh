#!/bin/bash
# Round 6: bf16 mode keeps x3 in bf16 (k_point_mlp<1> stores it, k_conv4_max
# copies it, the feature backward reads it).  The whole GPU suite, then the cls
# bench (configs[1], bf16 mode) alternated three times between the previous
# commit's tree (abhead/, its own package and library) and this tree, then a
# kernel trace of this tree's cls bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r06i}
root=$(pwd)
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread -rf > gpurun_out/${tag}_tests.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/${tag}_tests.log | tail -15
if [ $rc -ne 0 ]; then exit $rc; fi
for i in 1 2 3; do
  for v in A B; do
    if [ $v = A ]; then d=$root/abhead; else d=$root; fi
    (cd $d && timeout -k 10 200 python bench.py --config cls --steps 300 --warmup 30 --no-cpu) > gpurun_out/${tag}_cab_$v$i.log 2>&1 || { echo "bench $v failed"; tail -20 gpurun_out/${tag}_cab_$v$i.log; exit 1; }
    python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if '\"metric\"' in l][-1]); r=d.get('roofline', {}); print('$v', d['ms_per_step'], r.get('avg_launch_us'), r.get('pair', {}).get('avg_us'))" gpurun_out/${tag}_cab_$v$i.log
  done
done
rm -rf gpurun_out/${tag}_trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_trace -o run --output-format csv -- python bench.py --config cls --no-cpu --steps 20 --warmup 5 > gpurun_out/${tag}_trace.log 2>&1 || { echo "trace rc=$?"; exit 1; }
echo trace ok
