#!/bin/bash
# HIP runtime knobs (second sweep): cls bench under each setting, packet capture off as the base.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # run <tag> <config> <env...>
  local tag=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --config $cfg --steps 300 --warmup 30 --no-cpu > gpurun_out/env_$tag.log 2>&1 || { echo "bench $tag failed"; tail -5 gpurun_out/env_$tag.log; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if '\"metric\"' in l][-1]); print('$tag', '$*', d['ms_per_step'])" gpurun_out/env_$tag.log
}
P=DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
for i in 1 2; do
  run b$i cls $P
  run hdp$i cls $P DEBUG_CLR_KERNARG_HDP_FLUSH_WA=0
  run fgs0$i cls $P ROC_USE_FGS_KERNARG=0
  run fgs1$i cls $P ROC_USE_FGS_KERNARG=1
  run sss$i cls $P ROC_SYSTEM_SCOPE_SIGNAL=0
  run flush$i cls $P AMD_OPT_FLUSH=0
  run dd$i cls $P AMD_DIRECT_DISPATCH=0
  run skip$i cls $P ROC_SKIP_KERNEL_ARG_COPY=1
  run pc1hdp$i cls DEBUG_CLR_KERNARG_HDP_FLUSH_WA=0
done
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/env_trace_pc0 -o run --output-format csv -- python bench.py --no-cpu --config cls --steps 50 --warmup 10 > gpurun_out/env_trace.log 2>&1
