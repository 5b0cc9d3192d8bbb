#!/bin/bash
# The graphed trainer iteration as the step's launches alone (the batches
# gathered by the feature forward's first launch, the iteration epilogue in the
# finishing launch): the data / trainer / parity GPU tests, the trainer and adv
# benches, and a kernel trace of the trainer run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_data.py tests/test_gpu_distributed.py tests/test_gpu_g13.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/fold_tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/fold_tests.log)"; [ $rc -eq 0 ] || { grep -E "FAIL|Error|error" gpurun_out/fold_tests.log | head -20; exit $rc; }
for cfg in trainer adv; do
  timeout -k 10 300 python bench.py --config $cfg --no-cpu > gpurun_out/fold_$cfg.log 2>&1 || { echo "bench $cfg failed"; tail -5 gpurun_out/fold_$cfg.log; exit 1; }
  grep '"metric"' gpurun_out/fold_$cfg.log | tail -1 > gpurun_out/fold_$cfg.json
  python -c "import json; d=json.load(open('gpurun_out/fold_$cfg.json')); print('$cfg', d['ms_per_step'], 'replay', d.get('graph_replay_ms_per_step'), 'eager', d.get('eager_ms_per_step'))"
done
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/fold_trace -o run --output-format csv -- python bench.py --config trainer --no-cpu --steps 50 --warmup 10 --repeats 1 > gpurun_out/fold_trace.log 2>&1 || { echo "trace failed"; exit 1; }
