#!/bin/bash
# Seg: GPU seg tests, seg bench, kernel trace + conv6 PMC traffic.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_seg.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/s_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config seg --steps 20 --warmup 3 --no-cpu > gpurun_out/s_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep metric gpurun_out/s_bench.log | cut -c1-200
[ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/s_trace gpurun_out/s_pf gpurun_out/s_pw
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s_trace -o run --output-format csv -- python bench.py --config seg --no-cpu --steps 5 --warmup 1 > gpurun_out/s_trace.log 2>&1 || exit 1
python tools/kstats.py gpurun_out/s_trace/run_kernel_trace.csv > gpurun_out/s_kstats.txt; head -8 gpurun_out/s_kstats.txt
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/s_pf -o run --output-format csv -- python bench.py --config seg --no-cpu --steps 2 --warmup 1 > gpurun_out/s_pf.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/s_pw -o run --output-format csv -- python bench.py --config seg --no-cpu --steps 2 --warmup 1 > gpurun_out/s_pw.log 2>&1 || exit 1
python tools/pmc_traffic.py gpurun_out/s_pf gpurun_out/s_pw gpurun_out/s_traffic.json | grep -E "2, 2, 2, 3|max_combine"
