#!/bin/bash
# Copy one gpu_round.sh run's evidence from gpurun_out/ (scratch) into the
# tracked profiles/ directory: bench lines, kernel-trace summaries, PMC
# traffic summaries and one step's kernel timeline.  Runs on the CPU here.
set -euo pipefail
cd "$(dirname "$0")/.."
tag=${1:-r01}
o=gpurun_out
p=profiles
line() { grep '"metric"' "$1" | tail -1; }
line "$o/${tag}_bench.log" > "$p/${tag}_bench.json"
line "$o/${tag}_bench_seg.log" > "$p/${tag}_seg_bench.json"
line "$o/${tag}_bench_cls.log" > "$p/${tag}_cls_bench.json"
line "$o/${tag}_bench_n2048.log" > "$p/${tag}_bench_n2048.json"
cp "$o/${tag}_trace/run_kernel_stats.csv" "$p/${tag}_kernel_stats.csv"
cp "$o/${tag}_trace_seg/run_kernel_stats.csv" "$p/${tag}_seg_kernel_stats.csv"
python tools/kstats.py "$o/${tag}_trace/run_kernel_trace.csv" > "$p/${tag}_kernel_trace_summary.txt"
python tools/kstats.py "$o/${tag}_trace_seg/run_kernel_trace.csv" > "$p/${tag}_seg_kernel_trace_summary.txt"
python tools/step_timeline.py "$o/${tag}_trace/run_kernel_trace.csv" > "$p/${tag}_step_timeline.txt"
python tools/pmc_traffic.py "$o/${tag}_pmc_fetch" "$o/${tag}_pmc_write" "$p/${tag}_pmc_traffic.json" > /dev/null
python tools/pmc_traffic.py "$o/${tag}_pmc_fetch_seg" "$o/${tag}_pmc_write_seg" "$p/${tag}_seg_pmc_traffic.json" > /dev/null
cp "$o/${tag}_pytest.log" "$p/${tag}_pytest_gpu.log"
cp "$o/${tag}_smoke.log" "$p/${tag}_smoke.log"
echo "refreshed $p/${tag}_*"
