#!/bin/bash
# Round 6: the fused feature-transform cls step (ClsFtTrainStep, pcadv_cls_step
# part 3): its tests, the T-Net / FT / data tests, and cls_ft fused vs the
# autograd body (alternated twice) plus a kernel trace of the fused form.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r06h}
timeout -k 10 600 python -u -m pytest -v -s --timeout 200 --timeout-method thread tests/test_gpu_cls_ft_step.py tests/test_gpu_tnet.py tests/test_gpu_ft_step.py > gpurun_out/${tag}_tests.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/${tag}_tests.log | tail -15
if [ $rc -ne 0 ]; then exit $rc; fi
for rep in 1 2; do
  for f in 0 1; do
    a=""; [ $f = 0 ] && a="--ft-body"
    timeout -k 10 300 python bench.py --config cls_ft --no-cpu --steps 100 --warmup 10 $a > gpurun_out/${tag}_cls_ft_f${f}_${rep}.log 2>&1 || { echo "bench rc=$?"; tail -20 gpurun_out/${tag}_cls_ft_f${f}_${rep}.log; exit 1; }
    echo "cls_ft fused=$f rep=$rep $(grep -h '"metric"' gpurun_out/${tag}_cls_ft_f${f}_${rep}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  done
done
rm -rf gpurun_out/${tag}_trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_trace -o run --output-format csv -- python bench.py --config cls_ft --no-cpu --steps 20 --warmup 5 > gpurun_out/${tag}_trace.log 2>&1 || { echo "trace rc=$?"; exit 1; }
echo trace ok
