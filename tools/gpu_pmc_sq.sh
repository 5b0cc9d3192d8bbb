#!/bin/bash
# SQ instruction-mix / stall counter passes (one pass each) over one bench
# config's kernels; per kernel (name + grid) the mean of each counter over its
# launches.  usage: tools/gpu_pmc_sq.sh <tag> [bench.py args ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=$1; shift
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d gpurun_out/${tag}_sq$i -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu --repeats 1 "$@" > gpurun_out/${tag}_sq$i.log 2>&1
  rc=$?; echo "${tag}_sq$i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/${tag}_sq$i.log; exit $rc; fi
done
python tools/pmc_table.py gpurun_out/${tag}_sq1 gpurun_out/${tag}_sq2 > gpurun_out/${tag}_sq_table.txt
cat gpurun_out/${tag}_sq_table.txt
