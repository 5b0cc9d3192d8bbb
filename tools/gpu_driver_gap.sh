#!/bin/bash
# the driver's exact bench command beside a 200-step run on
# one lease, the in-process region probe (tools/driver_gap.py) and a kernel
# trace spanning the driver command's timed regions.
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
  echo "   rc=$rc"; grep -h '"metric"' "gpurun_out/${tag}_${name}.log" | cut -c1-400
  if [ $rc -ne 0 ]; then tail -20 "gpurun_out/${tag}_${name}.log"; exit $rc; fi
}
step drv1 300 python3 bench.py --gpus 1 --steps 20 --warmup 5
step s200a 300 python3 bench.py --gpus 1 --steps 200 --warmup 20 --no-cpu
step drv2 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu
step probe 300 python3 tools/driver_gap.py "gpurun_out/${tag}_driver_gap.json"
cat "gpurun_out/${tag}_driver_gap.json"
rm -rf "gpurun_out/${tag}_drvtrace"
step drvtrace 300 rocprofv3 --kernel-trace --stats -d "gpurun_out/${tag}_drvtrace" -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu
f=$(ls gpurun_out/${tag}_drvtrace/run_kernel_trace.csv gpurun_out/${tag}_drvtrace/*/*/run_kernel_trace.csv 2>/dev/null | head -1)
python3 tools/region_timeline.py "$f" > "gpurun_out/${tag}_driver_cmd_timeline.txt" && head -60 "gpurun_out/${tag}_driver_cmd_timeline.txt"
