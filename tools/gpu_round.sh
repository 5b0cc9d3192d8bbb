#!/bin/bash
# Round evidence on the GPU box: parity tests, smoke, a kernel-trace profile of
# each bench config, two PMC passes per config (FETCH_SIZE, WRITE_SIZE: they
# cannot share a pass on gfx950), and the bench lines (adv, seg, cls, adv at
# N=2048, the run_training loop).  Every GPU step has its own time limit; the
# script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r03}
only=${2:-all}
set -o pipefail

step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/${tag}_${name}.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -4 "gpurun_out/${tag}_${name}.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
prof() {  # prof <name> <bench args...>: kernel trace + the two PMC passes
  local name=$1; shift
  step trace$name 600 rocprofv3 --kernel-trace --stats -d "gpurun_out/${tag}_trace$name" -o run --output-format csv -- python bench.py --no-cpu "$@"
  step pmc_fetch$name 600 rocprofv3 --pmc FETCH_SIZE -d "gpurun_out/${tag}_pmc_fetch$name" -o run --output-format csv -- python bench.py --no-cpu --steps 3 --warmup 1 --repeats 1 "$@"
  step pmc_write$name 600 rocprofv3 --pmc WRITE_SIZE -d "gpurun_out/${tag}_pmc_write$name" -o run --output-format csv -- python bench.py --no-cpu --steps 3 --warmup 1 --repeats 1 "$@"
}

if [ "$only" = all ] || [ "$only" = tests ]; then
  step pytest 1500 python -u -m pytest tests -m gpu -v --timeout 900 --timeout-method thread -rf
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "$only" = all ] || [ "$only" = bench ]; then
  prof "" --steps 50 --warmup 10
  # the bench lines read their traffic from the summaries of these passes
  python tools/pmc_traffic.py "gpurun_out/${tag}_pmc_fetch" "gpurun_out/${tag}_pmc_write" "profiles/${tag}_pmc_traffic.json" > /dev/null
  prof _cls --config cls --steps 50 --warmup 10
  python tools/pmc_traffic.py "gpurun_out/${tag}_pmc_fetch_cls" "gpurun_out/${tag}_pmc_write_cls" "profiles/${tag}_cls_pmc_traffic.json" > /dev/null
  prof _seg --config seg --steps 5 --warmup 1
  python tools/pmc_traffic.py "gpurun_out/${tag}_pmc_fetch_seg" "gpurun_out/${tag}_pmc_write_seg" "profiles/${tag}_seg_pmc_traffic.json" > /dev/null
  step bench 600 python bench.py
  grep '"metric"' "gpurun_out/${tag}_bench.log"
  step bench_cls 600 python bench.py --config cls
  step bench_seg 600 python bench.py --config seg --steps 20 --warmup 3
  step bench_n2048 600 python bench.py --points 2048 --no-cpu --steps 100 --warmup 10
  step bench_trainer 600 python bench.py --config trainer --steps 300 --warmup 20
  step bench_cls_ft 600 python bench.py --config cls_ft --steps 100 --warmup 10
  step bench_adv_ft 600 python bench.py --config adv_ft --steps 100 --warmup 10
fi
if [ "$only" = all ] || [ "$only" = mfma ]; then
  bash tools/gpu_mfma.sh "$tag" || exit 1
fi
