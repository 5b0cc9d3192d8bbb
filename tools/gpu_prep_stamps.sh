#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python tools/tail_stamps.py > gpurun_out/ps_adv.log 2>&1 || { echo "adv stamps failed"; tail -5 gpurun_out/ps_adv.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ps_adv.log
timeout -k 10 120 python tools/tail_stamps.py cls > gpurun_out/ps_cls.log 2>&1 || { echo "cls stamps failed"; tail -5 gpurun_out/ps_cls.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ps_cls.log
