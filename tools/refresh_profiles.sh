#!/bin/bash
# Copy one gpu_round.sh run's evidence from gpurun_out/ (scratch) into the
# tracked profiles/ directory: bench lines, kernel-trace summaries, PMC
# traffic summaries and one step's kernel timeline.  Runs on the CPU here.
set -euo pipefail
cd "$(dirname "$0")/.."
tag=${1:-r03}
o=gpurun_out
p=profiles
line() { grep '"metric"' "$1" | tail -1; }
line "$o/${tag}_bench.log" > "$p/${tag}_bench.json"
line "$o/${tag}_bench_seg.log" > "$p/${tag}_seg_bench.json"
line "$o/${tag}_bench_cls.log" > "$p/${tag}_cls_bench.json"
line "$o/${tag}_bench_n2048.log" > "$p/${tag}_bench_n2048.json"
line "$o/${tag}_bench_trainer.log" > "$p/${tag}_trainer_bench.json"
for f in cls_ft adv_ft; do
  if [ -f "$o/${tag}_bench_$f.log" ]; then line "$o/${tag}_bench_$f.log" > "$p/${tag}_${f}_bench.json"; fi
done
for c in adv cls seg; do
  if [ -d "$o/${tag}_mfma_$c" ]; then
    python tools/pmc_mfma.py "$o/${tag}_mfma_$c" "$p/${tag}_${c}_mfma.json" "bench.py ($c)" > /dev/null
  fi
done
for c in "" _cls _seg; do
  cp "$o/${tag}_trace$c/run_kernel_stats.csv" "$p/${tag}${c}_kernel_stats.csv"
  python tools/kstats.py "$o/${tag}_trace$c/run_kernel_trace.csv" > "$p/${tag}${c}_kernel_trace_summary.txt"
  python tools/pmc_traffic.py "$o/${tag}_pmc_fetch$c" "$o/${tag}_pmc_write$c" "$p/${tag}${c}_pmc_traffic.json" > /dev/null
done
python tools/step_timeline.py "$o/${tag}_trace/run_kernel_trace.csv" > "$p/${tag}_step_timeline.txt"
python tools/step_timeline.py "$o/${tag}_trace_cls/run_kernel_trace.csv" > "$p/${tag}_cls_step_timeline.txt" || true
if [ -f "$o/${tag}_pytest.log" ]; then cp "$o/${tag}_pytest.log" "$p/${tag}_pytest_gpu.log"; fi
if [ -f "$o/${tag}_smoke.log" ]; then cp "$o/${tag}_smoke.log" "$p/${tag}_smoke.log"; fi
echo "refreshed $p/${tag}_*"
