#!/bin/bash
# Round 6: the chained point-wise forward (pcadv_pw_chain): its bitwise tests,
# the FT step / g13 / T-Net tests, then adv_ft and cls_ft A/B (per-layer
# launches vs chains, alternated twice).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r06d}
timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_pw_chain.py tests/test_gpu_ft_step.py tests/test_gpu_g13.py tests/test_gpu_tnet.py > gpurun_out/${tag}_tests.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/${tag}_tests.log | tail -15
if [ $rc -ne 0 ]; then tail -40 gpurun_out/${tag}_tests.log; exit $rc; fi
for rep in 1 2; do
  for ch in 0 1; do
    PCADV_FT_CHAIN=$ch timeout -k 10 300 python bench.py --config adv_ft --no-cpu --steps 100 --warmup 10 > gpurun_out/${tag}_adv_ft_c${ch}_${rep}.log 2>&1 || { echo "bench rc=$?"; tail -20 gpurun_out/${tag}_adv_ft_c${ch}_${rep}.log; exit 1; }
    echo "adv_ft chain=$ch rep=$rep $(grep -h '"metric"' gpurun_out/${tag}_adv_ft_c${ch}_${rep}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  done
done
rm -rf gpurun_out/${tag}_trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_trace -o run --output-format csv -- python bench.py --config adv_ft --no-cpu --steps 20 --warmup 5 > gpurun_out/${tag}_trace.log 2>&1 || { echo "trace rc=$?"; exit 1; }
echo trace ok
