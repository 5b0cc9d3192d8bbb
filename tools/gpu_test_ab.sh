cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/q_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/q_pytest.log; grep -E "FAIL|Error" gpurun_out/q_pytest.log | head -5
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab.sh
