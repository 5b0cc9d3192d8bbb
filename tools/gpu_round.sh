#!/bin/bash
# Round-end evidence on the GPU box: parity tests, a kernel-trace profile of
# the bench, two PMC passes (FETCH_SIZE, WRITE_SIZE: they cannot share a pass
# on gfx950) and the default bench line with its CPU baseline.  Every GPU step
# has its own time limit; the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r01}
set -o pipefail

step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/${tag}_${name}.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -4 "gpurun_out/${tag}_${name}.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
}

step pytest 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -rf
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step trace 600 rocprofv3 --kernel-trace --stats -d "gpurun_out/${tag}_trace" -o run --output-format csv -- python bench.py --no-cpu --steps 50 --warmup 10
step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d "gpurun_out/${tag}_pmc_fetch" -o run --output-format csv -- python bench.py --no-cpu --steps 3 --warmup 1
step pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d "gpurun_out/${tag}_pmc_write" -o run --output-format csv -- python bench.py --no-cpu --steps 3 --warmup 1
# the adv bench line reads its traffic from the summary of these passes
python tools/pmc_traffic.py "gpurun_out/${tag}_pmc_fetch" "gpurun_out/${tag}_pmc_write" "profiles/${tag}_pmc_traffic.json" > /dev/null
step bench 600 python bench.py
grep '"metric"' "gpurun_out/${tag}_bench.log"
step trace_seg 600 rocprofv3 --kernel-trace --stats -d "gpurun_out/${tag}_trace_seg" -o run --output-format csv -- python bench.py --config seg --no-cpu --steps 5 --warmup 1
step pmc_fetch_seg 600 rocprofv3 --pmc FETCH_SIZE -d "gpurun_out/${tag}_pmc_fetch_seg" -o run --output-format csv -- python bench.py --config seg --no-cpu --steps 2 --warmup 1
step pmc_write_seg 600 rocprofv3 --pmc WRITE_SIZE -d "gpurun_out/${tag}_pmc_write_seg" -o run --output-format csv -- python bench.py --config seg --no-cpu --steps 2 --warmup 1
# the seg bench line reads its traffic from the committed summary of these passes
python tools/pmc_traffic.py "gpurun_out/${tag}_pmc_fetch_seg" "gpurun_out/${tag}_pmc_write_seg" "profiles/${tag}_seg_pmc_traffic.json" > /dev/null
step bench_seg 600 python bench.py --config seg --steps 20 --warmup 3
step bench_cls 600 python bench.py --config cls
step bench_n2048 600 python bench.py --points 2048 --no-cpu --steps 100 --warmup 10
