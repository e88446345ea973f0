#!/bin/bash
# r6 session 14: the native high-priority 4-stream pool (HIPZAP_STREAM_KIND=hiprio) -- BERT 4 contexts
# fresh / after a 1-context engine; DP figures at depth 2 / 3 / 4 on it vs torch streams.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r6_s14
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_engine_streams_gpu.py > $OUT/tests.log 2>&1
rc=$?; tail -4 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for k in hiprio torch; do
    for m in fresh4 after1 after1_infer; do
      HIPZAP_STREAM_KIND=$k timeout -k 10 120 python3 -u scripts/diag_bert_iters.py --mode $m > $OUT/bert.tmp 2>$OUT/bert.err
      rc=$?; [ $rc -eq 0 ] || { tail -5 $OUT/bert.err; exit $rc; }
      echo "$k $(cat $OUT/bert.tmp)" | tee -a $OUT/summary.txt
    done
  done
done
P="python3 bench.py --cold-trials 0 --lm-cold 0 --bert-cold 0 --dyn-batch 0 --http-clients 0 --dp-figures 1 --config-figures 0 --cold-runs 0 --steps 40 --warmup 5 --sustained-s 0"
for d in 2 3 4; do
  for k in hiprio torch; do
    HIPZAP_DP_DEPTH=$d HIPZAP_STREAM_KIND=$k timeout -k 10 300 $P > $OUT/dp_${k}_$d.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { tail -5 $OUT/dp_${k}_$d.log; exit $rc; }
    grep '^{' $OUT/dp_${k}_$d.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); dp=d.get('dp_scatter') or {}; sh=dp.get('dp_shard_w8') or {}
print('$k depth $d gb32', (dp.get('resnet50_gb32') or {}).get('img_s'), 'vit', (dp.get('vit_b16_fp8_gb64') or {}).get('img_s'), 'bs4', (sh.get('resnet50_bs4') or {}).get('img_s_in_flight'), 'vit8', (sh.get('vit_b16_fp8_bs8') or {}).get('img_s_in_flight'))" | tee -a $OUT/summary.txt
  done
done
