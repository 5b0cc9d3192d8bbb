cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/d_trace
PCADV_LIB=build/stamps/libpcadv_stamps.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/d_trace -o run --output-format csv -- python bench.py --no-cpu --steps 30 --warmup 5 > gpurun_out/d_trace.log 2>&1
rc=$?; echo "trace rc=$rc"
python tools/kstats.py gpurun_out/d_trace/run_kernel_trace.csv | head -20
