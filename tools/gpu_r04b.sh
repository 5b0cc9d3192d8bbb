#!/bin/bash
# Round-4 check: the whole GPU suite, smoke, then the seg bench in both modes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r04b}
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread -rf > gpurun_out/${tag}_pytest.log 2>&1
rc=$?; tail -25 gpurun_out/${tag}_pytest.log | grep -E "passed|failed|FAILED|Error" ; echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/${tag}_smoke.log
timeout -k 10 300 python bench.py --config seg --steps 20 --warmup 3 --no-cpu > gpurun_out/${tag}_seg.log 2>&1 || exit $?
grep -o '"ms_per_step": [0-9.]*' gpurun_out/${tag}_seg.log
timeout -k 10 300 python bench.py --config seg --precision bf16 --steps 20 --warmup 3 --no-cpu > gpurun_out/${tag}_seg_bf.log 2>&1 || exit $?
grep -o '"ms_per_step": [0-9.]*' gpurun_out/${tag}_seg_bf.log
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu > gpurun_out/${tag}_adv.log 2>&1 || exit $?
grep -o '"ms_per_step": [0-9.]*' gpurun_out/${tag}_adv.log
timeout -k 10 120 python tools/fwd_stamps.py 64 1024 > gpurun_out/${tag}_stamps.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/${tag}_stamps.log | head -40
timeout -k 10 120 python tools/tail_stamps.py 32 1024 > gpurun_out/${tag}_tail_stamps.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/${tag}_tail_stamps.log | tail -30
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_trace -o run --output-format csv -- python bench.py --no-cpu --steps 50 --warmup 10 > gpurun_out/${tag}_trace.log 2>&1 || exit $?
python tools/kstats.py gpurun_out/${tag}_trace/run_kernel_trace.csv 2>/dev/null | head -20
