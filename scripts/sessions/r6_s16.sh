#!/bin/bash
# r6 session 16: the whole GPU test suite and smoke() as the driver runs them, then the headline on
# fresh high-priority streams vs torch's pool, then the default full bench.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r6_s16
mkdir -p $OUT
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -n 5 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
rc=$?; tail -n 2 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
B="python3 bench.py --cold-trials 0 --lm-cold 0 --bert-cold 0 --dyn-batch 0 --http-clients 0 --dp-figures 0 --config-figures 0 --cold-runs 0 --steps 20 --warmup 3"
for rep in 1 2; do
  for k in torch hiprio; do
    HIPZAP_STREAM_KIND=$k timeout -k 10 300 $B > $OUT/head_${k}_$rep.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { tail -n 5 $OUT/head_${k}_$rep.log; exit $rc; }
    grep '^{' $OUT/head_${k}_$rep.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print('$k rep $rep value', d['value'], 'sustained', (d.get('served_sustained') or {}).get('inf_s'), 'p50', d.get('latency_ms_p50_single'))" | tee -a $OUT/summary.txt
  done
done
