#!/bin/bash
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_seg.py -x -v --timeout 120 --timeout-method thread -k "256_tiles" > gpurun_out/big_t.log 2>&1
rc=$?; echo "big tests rc=$rc"; tail -8 gpurun_out/big_t.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest tests/test_gpu_seg.py -x -q --timeout 120 --timeout-method thread > gpurun_out/big_seg.log 2>&1
rc=$?; echo "seg tests rc=$rc"; tail -3 gpurun_out/big_seg.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in 0 1; do
    PCADV_GEMM_BIG=$v timeout -k 10 200 python bench.py --config seg --steps 20 --warmup 3 --no-cpu > gpurun_out/big_b$v$i.log 2>&1 || exit 1
    python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if '\"metric\"' in l][-1]); print('big=$v', d['ms_per_step'], d['roofline']['avg_launch_us'])" gpurun_out/big_b$v$i.log
  done
done
rm -rf gpurun_out/big_trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/big_trace -o run --output-format csv -- python bench.py --config seg --no-cpu --steps 5 --warmup 1 > gpurun_out/big_trace.log 2>&1 || exit 1
python tools/kstats.py gpurun_out/big_trace/run_kernel_trace.csv > gpurun_out/big_kstats.txt; head -14 gpurun_out/big_kstats.txt
