#!/bin/bash
# Round 6 evidence, second half: the MFMA-busy passes (adv, cls, seg) and the
# driver's exact bench command three times (fresh processes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_mfma.sh r06 || exit 1
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06_driver_cmd_$i.log 2>&1 || { echo "driver cmd rc=$?"; exit 1; }
  grep -h '"metric"' gpurun_out/r06_driver_cmd_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("driver cmd", d["ms_per_step"], d["timing"]["regions_s"])'
done
