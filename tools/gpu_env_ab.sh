#!/bin/bash
# HIP runtime knobs vs the graph-replayed step: cls and adv bench under each setting.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # run <tag> <config> <env...>
  local tag=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --config $cfg --steps 300 --warmup 30 --no-cpu > gpurun_out/env_$tag.log 2>&1 || { echo "bench $tag failed"; tail -5 gpurun_out/env_$tag.log; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if '\"metric\"' in l][-1]); print('$tag', '$*', d['ms_per_step'])" gpurun_out/env_$tag.log
}
for i in 1 2; do
  run cls_def$i cls X=1
  run cls_dk1$i cls HIP_FORCE_DEV_KERNARG=1
  run cls_dk0$i cls HIP_FORCE_DEV_KERNARG=0
  run cls_pc0$i cls DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
  run cls_pc1$i cls DEBUG_CLR_GRAPH_PACKET_CAPTURE=1
done
run adv_def adv X=1
run adv_dk1 adv HIP_FORCE_DEV_KERNARG=1
run adv_pc0 adv DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
