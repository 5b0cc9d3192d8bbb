#!/bin/bash
# Round 6: in-step stamps of the adversarial step (diagnostic library
# ablib/libstamps.so, `make stamps`): the tail kernels' phases, the chunk
# launch's chunk / dW4-gather / Adam workgroups, and the linear launches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r06n}
export PCADV_STAMPS_LIB=$(pwd)/ablib/libstamps.so
timeout -k 10 200 python tools/tail_stamps.py > gpurun_out/${tag}_tail_stamps.txt 2>&1 || { echo "tail stamps rc=$?"; tail -20 gpurun_out/${tag}_tail_stamps.txt; exit 1; }
timeout -k 10 200 python tools/lin_stamps.py > gpurun_out/${tag}_lin_stamps.txt 2>&1 || { echo "lin stamps rc=$?"; tail -20 gpurun_out/${tag}_lin_stamps.txt; exit 1; }
cat gpurun_out/${tag}_tail_stamps.txt gpurun_out/${tag}_lin_stamps.txt
