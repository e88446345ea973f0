#!/bin/bash
# r6 session 13: context streams from torch's normal-priority pool vs its high-priority pool
# (HIP: a separate set of 4 hardware queues per priority) vs dedicated CU-masked queues:
# BERT 4 contexts (fresh process, and after a 1-context engine), the DP figures, the headline.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r6_s13
mkdir -p $OUT
for rep in 1 2; do
  for k in torch hiprio cumask; do
    for m in fresh4 after1; do
      HIPZAP_STREAM_KIND=$k timeout -k 10 120 python3 -u scripts/diag_bert_iters.py --mode $m > $OUT/bert.tmp 2>$OUT/bert.err
      rc=$?; [ $rc -eq 0 ] || { tail -5 $OUT/bert.err; exit $rc; }
      echo "$k $(cat $OUT/bert.tmp)" | tee -a $OUT/summary.txt
    done
  done
done
P="python3 bench.py --cold-trials 0 --lm-cold 0 --bert-cold 0 --dyn-batch 0 --http-clients 0 --dp-figures 1 --config-figures 0 --cold-runs 0 --steps 40 --warmup 5 --sustained-s 2"
for rep in 1 2; do
  for k in torch hiprio; do
    HIPZAP_STREAM_KIND=$k timeout -k 10 300 $P > $OUT/dp_${k}_$rep.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { tail -5 $OUT/dp_${k}_$rep.log; exit $rc; }
    grep '^{' $OUT/dp_${k}_$rep.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); dp=d.get('dp_scatter') or {}; sh=dp.get('dp_shard_w8') or {}
print('$k rep $rep value', d['value'], 'sustained', (d.get('served_sustained') or {}).get('inf_s'), 'gb32', (dp.get('resnet50_gb32') or {}).get('img_s'), 'vit', (dp.get('vit_b16_fp8_gb64') or {}).get('img_s'), 'bs4', (sh.get('resnet50_bs4') or {}).get('img_s_in_flight'), 'vit8', (sh.get('vit_b16_fp8_bs8') or {}).get('img_s_in_flight'))" | tee -a $OUT/summary.txt
  done
done
