#!/bin/bash
# r6 session 25: fewer request streams (8 / 10 / 12) for the headline, interleaved.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r6_s25
mkdir -p $OUT
B="python3 bench.py --cold-trials 0 --lm-cold 0 --bert-cold 0 --dyn-batch 0 --http-clients 0 --dp-figures 0 --config-figures 0 --cold-runs 0 --steps 20 --warmup 3"
for rep in 1 2; do
  for s in 12 8 10; do
    timeout -k 10 300 $B --streams $s > $OUT/head_$s.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { tail -n 5 $OUT/head_$s.log; exit $rc; }
    grep '^{' $OUT/head_$s.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print('streams $s rep $rep value', d['value'], 'sustained', (d.get('served_sustained') or {}).get('inf_s'), 'p50', d.get('latency_ms_under_load_p50'), 'p99', d.get('latency_ms_under_load_p99'))" | tee -a $OUT/summary.txt
  done
done
