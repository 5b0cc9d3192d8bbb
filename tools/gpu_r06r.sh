#!/bin/bash
# Round 6: the chunk launch's ordered dispatch (long chunks, trailing items, short chunks).
# The conv4 / feature / step parity tests, then the adv bench (configs[2]) and
# the cls bench alternated three times between A = ablib/libA.so
# (-DPCADV_CHUNK_ORDER=0: chunks in cloud order) and B = this tree, then a kernel trace of B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r06r}
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/${tag}_tests.log | tail -15
if [ $rc -ne 0 ]; then exit $rc; fi
for i in 1 2 3; do
  for v in A B; do
    if [ $v = A ]; then lib=ablib/libA.so; else lib=adversarial_learning_on_pointclouds_amd/lib/libpcadv.so; fi
    PCADV_LIB=$lib timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu > gpurun_out/${tag}_adv_$v$i.log 2>&1 || { echo "bench $v failed"; tail -20 gpurun_out/${tag}_adv_$v$i.log; exit 1; }
    PCADV_LIB=$lib timeout -k 10 200 python bench.py --config cls --steps 300 --warmup 30 --no-cpu > gpurun_out/${tag}_cls_$v$i.log 2>&1 || { echo "bench cls $v failed"; tail -20 gpurun_out/${tag}_cls_$v$i.log; exit 1; }
    python -c "
import json,sys
def ln(f):
    d=json.loads([l for l in open(f) if '\"metric\"' in l][-1]); return d['ms_per_step'], d.get('roofline', {}).get('avg_launch_us')
print('$v adv', *ln(sys.argv[1]), 'cls', *ln(sys.argv[2]))" gpurun_out/${tag}_adv_$v$i.log gpurun_out/${tag}_cls_$v$i.log
  done
done
rm -rf gpurun_out/${tag}_trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_trace -o run --output-format csv -- python bench.py --no-cpu --steps 20 --warmup 5 > gpurun_out/${tag}_trace.log 2>&1 || { echo "trace rc=$?"; exit 1; }
echo trace ok
