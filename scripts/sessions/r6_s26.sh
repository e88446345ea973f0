#!/bin/bash
# r6 session 26: dynamic batching (6 contexts of batch 16) and the headline on fresh high-priority
# streams (HIPZAP_STREAM_KIND=hiprio) vs the default, interleaved.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r6_s26
mkdir -p $OUT
D="python3 bench.py --cold-trials 0 --lm-cold 0 --bert-cold 0 --http-clients 0 --dp-figures 0 --config-figures 0 --cold-runs 0 --steps 20 --warmup 3"
for rep in 1 2 3; do
  for k in auto hiprio; do
    HIPZAP_STREAM_KIND=$k timeout -k 10 300 $D > $OUT/dyn_$k.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { tail -n 5 $OUT/dyn_$k.log; exit $rc; }
    grep '^{' $OUT/dyn_$k.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); x=d.get('dynamic_batching') or {}
print('$k rep $rep value', d['value'], 'dyn', x.get('inf_s'), 'p50', x.get('latency_ms_p50'), 'p99', x.get('latency_ms_p99'))" | tee -a $OUT/summary.txt
  done
done
