#!/bin/bash
# Graph dispatch without packet capture (DEBUG_CLR_GRAPH_PACKET_CAPTURE=0): the GPU
# suite under it, then every bench config alternated default / pc0 twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 900 --timeout-method thread -rf -x > gpurun_out/pc0_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/pc0_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
run() {  # run <tag> <env> <bench args...>
  local tag=$1 e=$2; shift 2
  env $e timeout -k 10 300 python bench.py --no-cpu "$@" > gpurun_out/pc0_$tag.log 2>&1 || { echo "bench $tag failed"; tail -5 gpurun_out/pc0_$tag.log; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if '\"metric\"' in l][-1]); print('$tag', '$e', d['ms_per_step'])" gpurun_out/pc0_$tag.log
}
for i in 1 2; do
  for e in X=1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0; do
    t=${e%%=*}
    run adv_$t$i $e --steps 300 --warmup 30
    run cls_$t$i $e --config cls --steps 300 --warmup 30
    run trn_$t$i $e --config trainer --steps 300 --warmup 20
    run seg_$t$i $e --config seg --steps 20 --warmup 3
  done
done
