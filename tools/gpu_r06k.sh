#!/bin/bash
# Round 6: k_conv4_max's four-wave-group form for a bf16 x3 (cls, bf16 mode).
# The conv4 / bf16 parity tests, then the cls bench alternated three times
# between A = ablib/libA.so (-DPCADV_C4_G4=0: two wave groups, as before) and
# B = this tree, then a kernel trace of B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r06k}
timeout -k 10 600 python -u -m pytest -q --timeout 180 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_argmax_ties.py tests/test_gpu_data.py > gpurun_out/${tag}_tests.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/${tag}_tests.log | tail -15
if [ $rc -ne 0 ]; then exit $rc; fi
for i in 1 2 3; do
  for v in A B; do
    if [ $v = A ]; then lib=ablib/libA.so; else lib=adversarial_learning_on_pointclouds_amd/lib/libpcadv.so; fi
    PCADV_LIB=$lib timeout -k 10 200 python bench.py --config cls --steps 300 --warmup 30 --no-cpu > gpurun_out/${tag}_$v$i.log 2>&1 || { echo "bench $v failed"; tail -20 gpurun_out/${tag}_$v$i.log; exit 1; }
    python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if '\"metric\"' in l][-1]); r=d.get('roofline', {}); print('$v', d['ms_per_step'], r.get('avg_launch_us'), r.get('pair', {}).get('avg_us'))" gpurun_out/${tag}_$v$i.log
  done
done
rm -rf gpurun_out/${tag}_trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_trace -o run --output-format csv -- python bench.py --config cls --no-cpu --steps 20 --warmup 5 > gpurun_out/${tag}_trace.log 2>&1 || { echo "trace rc=$?"; exit 1; }
echo trace ok
