#!/bin/bash
# A/B of the cls FT step (point-wise kernels): the tree library against
# build/abx/lib*.so, after the T-Net / data GPU tests on the tree library;
# alternated 3x on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
tree=adversarial_learning_on_pointclouds_amd/lib/libpcadv.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_tnet.py tests/test_gpu_data.py -k "not seg" > gpurun_out/pw_tests.log 2>&1 || { tail -20 gpurun_out/pw_tests.log; exit 1; }
tail -1 gpurun_out/pw_tests.log
for i in 1 2 3; do
  for lib in build/abx/lib*.so $tree; do
    PCADV_LIB=$lib timeout -k 10 200 python bench.py --config cls_ft --steps 200 --warmup 20 --no-cpu > gpurun_out/pw_ab.json 2>/dev/null || { echo "bench failed"; exit 1; }
    python -c "import json,sys; d=json.loads(open('gpurun_out/pw_ab.json').read().strip().splitlines()[-1]); print('AB', sys.argv[1], d['ms_per_step'])" $(basename $lib)
  done
done
