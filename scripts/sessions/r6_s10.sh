#!/bin/bash
# r6 session 10: context streams from torch's pool vs fresh HIP streams vs full-CU-mask streams
# (HIPZAP_STREAM_KIND): BERT 4 contexts (fresh process each) and the ResNet-50 headline, interleaved.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r6_s10
mkdir -p $OUT
for rep in 1 2; do
  for k in torch native cumask; do
    HIPZAP_STREAM_KIND=$k timeout -k 10 120 python3 -u scripts/diag_bert_iters.py --mode fresh4 > $OUT/bert_$k.tmp 2>$OUT/bert_$k.err
    rc=$?; [ $rc -eq 0 ] || { tail -5 $OUT/bert_$k.err; exit $rc; }
    echo "$k $(cat $OUT/bert_$k.tmp)" | tee -a $OUT/bert_kinds.txt
  done
done
B="python3 bench.py --cold-trials 0 --lm-cold 0 --bert-cold 0 --dyn-batch 0 --http-clients 0 --dp-figures 0 --config-figures 0 --cold-runs 0 --steps 20 --warmup 3"
for rep in 1 2; do
  for k in torch native cumask; do
    HIPZAP_STREAM_KIND=$k timeout -k 10 300 $B > $OUT/head_${k}_$rep.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { tail -5 $OUT/head_${k}_$rep.log; exit $rc; }
    grep '^{' $OUT/head_${k}_$rep.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('$k rep $rep value', d['value'], 'sustained', json.dumps(d.get('served_sustained'))[:120], 'p50', d.get('latency_ms_p50_single'), 'single', d.get('single_stream_inf_s'), 'pipelined', d.get('device_pipelined_inf_s'))" | tee -a $OUT/head_kinds.txt
  done
done
