cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/cls_pytest.log 2>&1 || { tail -5 gpurun_out/cls_pytest.log; exit 1; }
tail -1 gpurun_out/cls_pytest.log
bash tools/gpu_cls_ab.sh || exit 1
rm -rf gpurun_out/cls_trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/cls_trace -o run --output-format csv -- python bench.py --config cls --no-cpu --steps 30 --warmup 5 > gpurun_out/cls_trace.log 2>&1 || exit 1
python tools/step_timeline.py gpurun_out/cls_trace/run_kernel_trace.csv > gpurun_out/cls_timeline.txt; cat gpurun_out/cls_timeline.txt
