#!/bin/bash
# MFMA-utilisation evidence: one rocprofv3 pass per bench
# config with the matrix-pipe busy counter, GPU-busy cycles and the kernel trace
# of the same dispatches; tools/pmc_mfma.py writes profiles/<tag>_<cfg>_mfma.json.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r05}
set -o pipefail
CTRS="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE"
for cfg in adv cls seg; do
  case $cfg in
    adv) args="--steps 3 --warmup 1" ;;
    cls) args="--config cls --steps 3 --warmup 1" ;;
    seg) args="--config seg --steps 2 --warmup 1" ;;
  esac
  d=gpurun_out/${tag}_mfma_$cfg
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $CTRS -d $d -o run --output-format csv -- \
    python bench.py --no-cpu --repeats 1 $args > $d.log 2>&1
  rc=$?; echo "mfma $cfg rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $d.log; exit $rc; fi
  python tools/pmc_mfma.py $d gpurun_out/${tag}_${cfg}_mfma.json "python bench.py $args" || exit 1
done
