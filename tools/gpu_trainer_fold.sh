#!/bin/bash
# The graphed trainer iteration with one gather launch for both loaders and the
# iteration epilogue folded into the step's finishing launch: the data / trainer
# GPU tests, the trainer bench, and a kernel trace of the trainer run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_data.py tests/test_gpu_distributed.py tests/test_gpu_g13.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/fold_tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/fold_tests.log)"; [ $rc -eq 0 ] || { grep -E "FAIL|Error|error" gpurun_out/fold_tests.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --config trainer --no-cpu > gpurun_out/fold_trainer.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/fold_trainer.log; exit 1; }
grep '"metric"' gpurun_out/fold_trainer.log | tail -1 > gpurun_out/fold_trainer.json
python -c "import json; d=json.load(open('gpurun_out/fold_trainer.json')); print('trainer', d['ms_per_step'], 'replay', d.get('graph_replay_ms_per_step'), 'eager', d.get('eager_ms_per_step'))"
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/fold_trace -o run --output-format csv -- python bench.py --config trainer --no-cpu --steps 50 --warmup 10 --repeats 1 > gpurun_out/fold_trace.log 2>&1 || { echo "trace failed"; exit 1; }
