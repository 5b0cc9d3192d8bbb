#!/bin/bash
# Steps per graph replay: adv and cls benches at 1 / 2 / 4 steps per graph, alternated twice;
# then a kernel trace of the adv bench at 4 (inter-step gaps).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {
  local tag=$1; shift
  timeout -k 10 300 python bench.py --no-cpu "$@" > gpurun_out/gs_$tag.log 2>&1 || { echo "bench $tag failed"; tail -5 gpurun_out/gs_$tag.log; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if '\"metric\"' in l][-1]); print('$tag', d['ms_per_step'], d['config'].get('steps_per_graph'))" gpurun_out/gs_$tag.log
}
for i in 1 2; do
  for g in 1 2 4; do
    run adv_g$g_$i --steps 400 --warmup 40 --graph-steps $g
    run cls_g$g_$i --config cls --steps 400 --warmup 40 --graph-steps $g
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/gs_trace -o run --output-format csv -- python bench.py --no-cpu --steps 40 --warmup 8 --graph-steps 4 > gpurun_out/gs_trace.log 2>&1
