#!/bin/bash
# Round 6: the seg forward's weights split once per step (pcadv_split_bf3 +
# pcadv_gemm_b3): bitwise tests, the seg suite, then seg A/B (PCADV_SEG_B3=1 vs 0)
# alternated twice, and a kernel trace of the new form.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r06e}
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_seg.py > gpurun_out/${tag}_tests.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/${tag}_tests.log | tail -15
if [ $rc -ne 0 ]; then tail -40 gpurun_out/${tag}_tests.log; exit $rc; fi
for rep in 1 2; do
  for b in 0 1; do
    PCADV_SEG_B3=$b timeout -k 10 300 python bench.py --config seg --no-cpu --steps 20 --warmup 3 > gpurun_out/${tag}_seg_b${b}_${rep}.log 2>&1 || { echo "bench rc=$?"; tail -20 gpurun_out/${tag}_seg_b${b}_${rep}.log; exit 1; }
    echo "seg b3=$b rep=$rep $(grep -h '"metric"' gpurun_out/${tag}_seg_b${b}_${rep}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  done
done
rm -rf gpurun_out/${tag}_trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_trace -o run --output-format csv -- python bench.py --config seg --no-cpu --steps 5 --warmup 1 > gpurun_out/${tag}_trace.log 2>&1 || { echo "trace rc=$?"; exit 1; }
echo trace ok
