#!/bin/bash
# Round 6: evidence for the fused feature-transform step (kernel trace, two
# PMC traffic passes, the MFMA-busy pass) and the cls step's timeline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r06}
set -o pipefail
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/${tag}_${name}.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; grep -h '"metric"' "gpurun_out/${tag}_${name}.log" | cut -c1-300
  if [ $rc -ne 0 ]; then tail -20 "gpurun_out/${tag}_${name}.log"; exit $rc; fi
}
A="--config adv_ft --no-cpu"
rm -rf gpurun_out/${tag}_trace_adv_ft gpurun_out/${tag}_pmc_fetch_adv_ft gpurun_out/${tag}_pmc_write_adv_ft gpurun_out/${tag}_mfma_adv_ft
step trace_adv_ft 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_trace_adv_ft -o run --output-format csv -- python bench.py $A --steps 20 --warmup 5
step pmc_fetch_adv_ft 150 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${tag}_pmc_fetch_adv_ft -o run --output-format csv -- python bench.py $A --steps 3 --warmup 1 --repeats 1
step pmc_write_adv_ft 150 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${tag}_pmc_write_adv_ft -o run --output-format csv -- python bench.py $A --steps 3 --warmup 1 --repeats 1
python tools/pmc_traffic.py gpurun_out/${tag}_pmc_fetch_adv_ft gpurun_out/${tag}_pmc_write_adv_ft profiles/${tag}_adv_ft_pmc_traffic.json > /dev/null || exit 1
CTRS="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE"
step mfma_adv_ft 150 rocprofv3 --kernel-trace --pmc $CTRS -d gpurun_out/${tag}_mfma_adv_ft -o run --output-format csv -- python bench.py $A --steps 3 --warmup 1 --repeats 1
python tools/pmc_mfma.py gpurun_out/${tag}_mfma_adv_ft profiles/${tag}_adv_ft_mfma.json "python bench.py $A --steps 3 --warmup 1" || exit 1
rm -rf gpurun_out/${tag}_trace_cls
step trace_cls 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_trace_cls -o run --output-format csv -- python bench.py --config cls --no-cpu --steps 20 --warmup 5
python tools/region_timeline.py gpurun_out/${tag}_trace_cls/run_kernel_trace.csv > gpurun_out/${tag}_cls_region_timeline.txt || exit 1
step adv_ft 300 python bench.py --config adv_ft --steps 100 --warmup 10
