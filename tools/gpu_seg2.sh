set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
PCADV_SEG_DGRAD_PRECISE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_seg.py -x -q --timeout 120 --timeout-method thread > gpurun_out/seg_tests_p.log 2>&1; tail -2 gpurun_out/seg_tests_p.log
bash tools/gpu_seg.sh
