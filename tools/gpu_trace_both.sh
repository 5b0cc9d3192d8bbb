#!/bin/bash
# Kernel trace + one step's timeline of the adv and cls benches (this tree).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in adv cls; do
  rm -rf gpurun_out/tr_$cfg
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tr_$cfg -o run --output-format csv -- python bench.py --config $cfg --no-cpu --steps 30 --warmup 5 > gpurun_out/tr_$cfg.log 2>&1 || { echo "trace $cfg failed"; exit 1; }
  python tools/step_timeline.py gpurun_out/tr_$cfg/run_kernel_trace.csv > gpurun_out/tr_${cfg}_timeline.txt; cat gpurun_out/tr_${cfg}_timeline.txt
done
