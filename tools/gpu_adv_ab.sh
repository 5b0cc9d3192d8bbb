#!/bin/bash
# Adv A/B against build/ab/libA.so (A = a previous tree's library, B = this
# tree's): the GPU suite on this tree, then the adv bench alternated three
# times, then a kernel trace + one step's timeline of B.  Each GPU step has its
# own time limit; the first failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/aab_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/aab_pytest.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for v in A B; do
    if [ $v = A ]; then lib=build/ab/libA.so; else lib=adversarial_learning_on_pointclouds_amd/lib/libpcadv.so; fi
    PCADV_LIB=$lib timeout -k 10 200 python bench.py --steps 300 --warmup 30 --no-cpu > gpurun_out/aab_$v$i.log 2>&1 || { echo "bench $v failed"; exit 1; }
    python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if '\"metric\"' in l][-1]); print('$v', d['ms_per_step'], d['roofline']['avg_launch_us'])" gpurun_out/aab_$v$i.log
  done
done
rm -rf gpurun_out/aab_trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/aab_trace -o run --output-format csv -- python bench.py --no-cpu --steps 30 --warmup 5 > gpurun_out/aab_trace.log 2>&1 || exit 1
python tools/kstats.py gpurun_out/aab_trace/run_kernel_trace.csv > gpurun_out/aab_kstats.txt; head -16 gpurun_out/aab_kstats.txt
python tools/step_timeline.py gpurun_out/aab_trace/run_kernel_trace.csv > gpurun_out/aab_timeline.txt; cat gpurun_out/aab_timeline.txt
