#!/bin/bash
# Same-box interleaved A/B of two native builds: base = hipzap/_lib/ab/libhipzap_base.so (an older
# tree compiled by hand), new = the in-tree hipzap/_lib/libhipzap.so.
#   CMD="python scripts/bench_models.py bert-base" REPS=2 bash scripts/ab_lib.sh
set -u
OUT=${OUT:-gpurun_out/ab_lib}
mkdir -p $OUT
for rep in $(seq 1 ${REPS:-2}); do
  for v in base new; do
    log=$OUT/${v}_$rep.log
    if [ $v = base ]; then export HIPZAP_LIB=hipzap/_lib/ab/libhipzap_base.so; else unset HIPZAP_LIB; fi
    timeout -k 10 ${TMO:-300} $CMD > $log 2>&1
    rc=$?
    echo "$v rep$rep rc=$rc $(grep -h '^{' $log | python3 -c 'import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d.get("model"), d.get("contexts", d.get("streams_per_gpu")), d.get("items_per_s", d.get("value")), end=" | ")' 2>/dev/null)"
    if [ $rc -ne 0 ]; then echo "STOP $v rc=$rc"; tail -5 $log; exit $rc; fi
  done
done
