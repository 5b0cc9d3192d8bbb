export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread -rf -k "bf16 or workgroup_forms or conv4_max_alone" > gpurun_out/r03e_pytest.log 2>&1; tail -3 gpurun_out/r03e_pytest.log
bash tools/gpu_cls_ab.sh
