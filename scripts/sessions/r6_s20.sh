#!/bin/bash
# r6 session 20: request streams per GPU for the headline (12 / 16 / 20 / 24) and the dynamic-
# batching shape (replay batch 16 / 32, contexts 6 / 8), interleaved, on the final program.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r6_s20
mkdir -p $OUT
B="python3 bench.py --cold-trials 0 --lm-cold 0 --bert-cold 0 --dyn-batch 0 --http-clients 0 --dp-figures 0 --config-figures 0 --cold-runs 0 --steps 20 --warmup 3"
for rep in 1 2; do
  for s in 16 12 20 24; do
    timeout -k 10 300 $B --streams $s > $OUT/head_$s.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { tail -n 5 $OUT/head_$s.log; exit $rc; }
    grep '^{' $OUT/head_$s.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print('streams $s rep $rep value', d['value'], 'sustained', (d.get('served_sustained') or {}).get('inf_s'), 'p50', d.get('latency_ms_under_load_p50'), 'p99', d.get('latency_ms_under_load_p99'))" | tee -a $OUT/summary.txt
  done
done
D="python3 bench.py --cold-trials 0 --lm-cold 0 --bert-cold 0 --http-clients 0 --dp-figures 0 --config-figures 0 --cold-runs 0 --steps 5 --warmup 2 --sustained-s 0"
for rep in 1 2; do
  for cfg in "16 6" "16 8" "32 4" "32 6"; do
    set -- $cfg
    timeout -k 10 300 $D --dyn-batch $1 --dyn-contexts $2 > $OUT/dyn.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { tail -n 5 $OUT/dyn.log; exit $rc; }
    grep '^{' $OUT/dyn.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); x=d.get('dynamic_batching') or {}
print('dyn batch $1 contexts $2 rep $rep', x.get('inf_s'), 'p50', x.get('latency_ms_p50'), 'p99', x.get('latency_ms_p99'))" | tee -a $OUT/summary.txt
  done
done
