#!/bin/bash
# The GPU suite, then kernel traces + one step's timeline of the adv, cls and
# seg benches (this tree).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/st_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/st_pytest.log
[ $rc -eq 0 ] || exit $rc
for cfg in adv cls seg; do
  rm -rf gpurun_out/tr_$cfg
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tr_$cfg -o run --output-format csv -- python bench.py --config $cfg --no-cpu --steps 20 --warmup 5 > gpurun_out/tr_$cfg.log 2>&1 || { echo "trace $cfg failed"; exit 1; }
  python tools/step_timeline.py gpurun_out/tr_$cfg/run_kernel_trace.csv > gpurun_out/tr_${cfg}_timeline.txt
  tail -1 gpurun_out/tr_${cfg}_timeline.txt
done
cat gpurun_out/tr_cls_timeline.txt
