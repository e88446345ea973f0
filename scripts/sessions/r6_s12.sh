#!/bin/bash
# r6 session 12: the bs=1 headline with fewer request streams on dedicated hardware queues
# (HIPZAP_STREAM_KIND=cumask) vs torch's pooled streams; and dynamic batching over 4 dedicated-queue
# contexts vs 6 pooled ones.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r6_s12
mkdir -p $OUT
B="python3 bench.py --cold-trials 0 --lm-cold 0 --bert-cold 0 --dyn-batch 0 --http-clients 0 --dp-figures 0 --config-figures 0 --cold-runs 0 --steps 20 --warmup 3"
for rep in 1 2; do
  for cfg in "torch 16" "cumask 4" "torch 4" "cumask 6" "torch 8"; do
    set -- $cfg
    HIPZAP_STREAM_KIND=$1 timeout -k 10 300 $B --streams $2 > $OUT/head_$1_$2_$rep.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { tail -5 $OUT/head_$1_$2_$rep.log; exit $rc; }
    grep '^{' $OUT/head_$1_$2_$rep.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print('$1 streams $2 rep $rep value', d['value'], 'sustained', (d.get('served_sustained') or {}).get('inf_s'), 'p50_load', d.get('latency_ms_under_load_p50'), 'p99_load', d.get('latency_ms_under_load_p99'), 'pipelined', d.get('device_pipelined_inf_s'))" | tee -a $OUT/summary.txt
  done
done
D="python3 bench.py --cold-trials 0 --lm-cold 0 --bert-cold 0 --http-clients 0 --dp-figures 0 --config-figures 0 --cold-runs 0 --steps 5 --warmup 2 --sustained-s 0 --dyn-batch 16"
for rep in 1 2; do
  for cfg in "auto 6" "auto 4" "torch 4"; do
    set -- $cfg
    HIPZAP_STREAM_KIND=$1 timeout -k 10 300 $D --dyn-contexts $2 > $OUT/dyn_$1_$2_$rep.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { tail -5 $OUT/dyn_$1_$2_$rep.log; exit $rc; }
    grep '^{' $OUT/dyn_$1_$2_$rep.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); x=d.get('dynamic_batching') or {}
print('dyn $1 contexts $2 rep $rep', x.get('inf_s'), 'p50', x.get('latency_ms_p50'), 'p99', x.get('latency_ms_p99'))" | tee -a $OUT/summary.txt
  done
done
P="python3 bench.py --cold-trials 0 --lm-cold 0 --bert-cold 0 --dyn-batch 0 --http-clients 0 --dp-figures 1 --config-figures 0 --cold-runs 0 --steps 40 --warmup 5 --sustained-s 0"
for rep in 1 2; do
  for k in auto torch; do
    HIPZAP_STREAM_KIND=$k timeout -k 10 300 $P > $OUT/dp_${k}_$rep.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { tail -5 $OUT/dp_${k}_$rep.log; exit $rc; }
    grep '^{' $OUT/dp_${k}_$rep.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); dp=d.get('dp_scatter') or {}; sh=dp.get('dp_shard_w8') or {}
print('dp $k rep $rep gb32', (dp.get('resnet50_gb32') or {}).get('img_s'), 'one', (dp.get('resnet50_gb32') or {}).get('img_s_one_in_flight'), 'vit', (dp.get('vit_b16_fp8_gb64') or {}).get('img_s'), 'bs4', (sh.get('resnet50_bs4') or {}).get('img_s_in_flight'), 'vit8', (sh.get('vit_b16_fp8_bs8') or {}).get('img_s_in_flight'))" | tee -a $OUT/summary.txt
  done
done
