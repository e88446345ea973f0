#!/bin/bash
# r6 session 15: auto = fresh high-priority streams for every 2-4-context engine vs torch's pool:
# BERT 4 contexts (fresh / after a 1-context engine), DP figures at the default depths and at 3.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r6_s15
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_engine_streams_gpu.py tests/test_dp_gpu.py > $OUT/tests.log 2>&1
rc=$?; tail -4 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for k in auto torch; do
    for m in fresh4 after1 after1_infer; do
      HIPZAP_STREAM_KIND=$k timeout -k 10 120 python3 -u scripts/diag_bert_iters.py --mode $m > $OUT/bert.tmp 2>$OUT/bert.err
      rc=$?; [ $rc -eq 0 ] || { tail -5 $OUT/bert.err; exit $rc; }
      echo "$k $(cat $OUT/bert.tmp)" | tee -a $OUT/summary.txt
    done
  done
done
P="python3 bench.py --cold-trials 0 --lm-cold 0 --bert-cold 0 --dyn-batch 0 --http-clients 0 --dp-figures 1 --config-figures 0 --cold-runs 0 --steps 40 --warmup 5 --sustained-s 0"
for cfg in "auto 0" "torch 0" "auto 3" "torch 3" "auto 0" "torch 0"; do
  set -- $cfg
  if [ $2 = 0 ]; then unset HIPZAP_DP_DEPTH; else export HIPZAP_DP_DEPTH=$2; fi
  HIPZAP_STREAM_KIND=$1 timeout -k 10 300 $P > $OUT/dp.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { tail -5 $OUT/dp.log; exit $rc; }
  grep '^{' $OUT/dp.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); dp=d.get('dp_scatter') or {}; sh=dp.get('dp_shard_w8') or {}
print('$1 depth $2 gb32', (dp.get('resnet50_gb32') or {}).get('img_s'), 'vit', (dp.get('vit_b16_fp8_gb64') or {}).get('img_s'), 'bs4', (sh.get('resnet50_bs4') or {}).get('img_s_in_flight'), 'vit8', (sh.get('vit_b16_fp8_bs8') or {}).get('img_s_in_flight'))" | tee -a $OUT/summary.txt
done
unset HIPZAP_DP_DEPTH
