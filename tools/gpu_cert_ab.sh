#!/bin/bash
# what certifying k_conv4_max's argmax costs.  A/B of the
# product library against -DPCADV_C4_CERT=1 (third-candidate tracking only),
# alternated three times, then the flag counts of -DPCADV_C4_CERT=2
# (tools/cert_diag.py).  Diagnostic libraries only; the product never loads them.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r06_cert}
set -o pipefail
for i in 1 2 3; do
  for v in prod cert1; do
    if [ $v = prod ]; then unset PCADV_LIB; else export PCADV_LIB=build/cert/lib$v.so; fi
    timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu > gpurun_out/${tag}_${v}_$i.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { tail -20 gpurun_out/${tag}_${v}_$i.log; exit $rc; }
    python - "$v" "$i" gpurun_out/${tag}_${v}_$i.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[3]) if l.startswith("{")][-1])
print(sys.argv[1], sys.argv[2], "ms/step", d["ms_per_step"], "conv4 us", d["roofline"]["avg_launch_us"], "pair us", d["roofline"]["pair"]["avg_us"])
PY
  done
done
export PCADV_LIB=build/cert/libcert2.so
timeout -k 10 300 python tools/cert_diag.py gpurun_out/${tag}_counts.json > gpurun_out/${tag}_counts.log 2>&1
rc=$?; tail -40 gpurun_out/${tag}_counts.log; exit $rc
