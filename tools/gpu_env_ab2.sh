#!/bin/bash
# More HIP runtime knobs vs the graph-replayed adversarial step (alternated twice).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # run <tag> <env...>
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 300 --warmup 30 --no-cpu > gpurun_out/env2_$tag.log 2>&1 || { echo "bench $tag failed"; tail -5 gpurun_out/env2_$tag.log; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if '\"metric\"' in l][-1]); print('$tag', '$*', d['ms_per_step'])" gpurun_out/env2_$tag.log
}
for i in 1 2; do
  run def$i X=1
  run optflush1_$i AMD_OPT_FLUSH=1
  run optflush0_$i AMD_OPT_FLUSH=0
  run flushexec0_$i GPU_FLUSH_ON_EXECUTION=0
  run graphq1_$i DEBUG_HIP_FORCE_GRAPH_QUEUES=1
  run kcopy0_$i DEBUG_HIP_KERNARG_COPY_OPT=0
done
