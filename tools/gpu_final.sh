#!/bin/bash
# Round-end evidence in two gpurun calls (each under the 20-minute limit):
#   bash tools/gpu_final.sh <tag> A   the whole -m gpu suite, smoke(), the
#        MFMA-busy passes and, per bench config (adv, cls, seg), a kernel trace
#        and the two PMC traffic passes
#   bash tools/gpu_final.sh <tag> B   every bench line (they read the PMC
#        summaries tools/refresh_profiles.sh wrote into profiles/ from call A)
#        and the driver's exact command three times
# Every GPU step has its own time limit; the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:?tag}
part=${2:?A or B}
set -o pipefail

step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/${tag}_${name}.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -3 "gpurun_out/${tag}_${name}.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
prof() {  # prof <name> <bench args...>: kernel trace + the two PMC passes
  local name=$1; shift
  step trace$name 300 rocprofv3 --kernel-trace --stats -d "gpurun_out/${tag}_trace$name" -o run --output-format csv -- python bench.py --no-cpu "$@"
  step pmc_fetch$name 300 rocprofv3 --pmc FETCH_SIZE -d "gpurun_out/${tag}_pmc_fetch$name" -o run --output-format csv -- python bench.py --no-cpu --steps 3 --warmup 1 --repeats 1 "$@"
  step pmc_write$name 300 rocprofv3 --pmc WRITE_SIZE -d "gpurun_out/${tag}_pmc_write$name" -o run --output-format csv -- python bench.py --no-cpu --steps 3 --warmup 1 --repeats 1 "$@"
}

if [ "$part" = A ]; then
  step pytest 600 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread -rf
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
  bash tools/gpu_mfma.sh "$tag" || exit 1
  prof "" --steps 50 --warmup 10
  prof _cls --config cls --steps 50 --warmup 10
  prof _seg --config seg --steps 5 --warmup 1
  prof _adv_ft --config adv_ft --steps 20 --warmup 5
fi
if [ "$part" = B ]; then
  step bench 300 python bench.py
  step bench_cls 300 python bench.py --config cls
  step bench_seg 300 python bench.py --config seg --steps 20 --warmup 3
  step bench_n2048 300 python bench.py --points 2048 --no-cpu --steps 100 --warmup 10
  step bench_trainer 300 python bench.py --config trainer --steps 300 --warmup 20
  step bench_cls_ft 300 python bench.py --config cls_ft --steps 100 --warmup 10
  step bench_adv_ft 300 python bench.py --config adv_ft --steps 100 --warmup 10
  for i in 1 2 3; do
    step driver_cmd_$i 300 python bench.py --gpus 1 --steps 20 --warmup 5
  done
  grep -h '"metric"' gpurun_out/${tag}_bench*.log gpurun_out/${tag}_driver_cmd_*.log | python -c '
import json, sys
for l in sys.stdin:
    d = json.loads(l)
    print(d["metric"][:60], d["ms_per_step"], d["value"])'
fi
