#!/bin/bash
# bf16 x3 copy handed from k_point_mlp to k_conv4_max: parity tests touching the feature
# forward and cls, then the cls bench A/B (build/ab/libA.so = before).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -k "conv4 or feat or cls or bf16 or smoke" --timeout 600 --timeout-method thread -rf -x > gpurun_out/r03k_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r03k_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_cls_ab.sh
