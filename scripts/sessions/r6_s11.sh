#!/bin/bash
# r6 session 11: dedicated hardware queues for 2-4-context engines (HIPZAP_STREAM_KIND=auto) --
# the stream test, then config figures and DP figures with auto vs torch streams, interleaved.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r6_s11
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_engine_streams_gpu.py tests/test_dp_gpu.py > $OUT/tests.log 2>&1
rc=$?; tail -9 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
B="python3 bench.py --cold-trials 0 --lm-cold 0 --bert-cold 0 --dyn-batch 16 --http-clients 0 --dp-figures 1 --config-figures 1 --cold-runs 0 --steps 40 --warmup 5 --sustained-s 0"
for rep in 1 2; do
  for k in auto torch; do
    HIPZAP_STREAM_KIND=$k timeout -k 10 400 $B > $OUT/bench_${k}_$rep.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { tail -5 $OUT/bench_${k}_$rep.log; exit $rc; }
    grep '^{' $OUT/bench_${k}_$rep.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); dp=d.get('dp_scatter') or {}; c=d.get('configs') or {}
sh=dp.get('dp_shard_w8') or {}
print('$k rep $rep value', d['value'], 'dyn', (d.get('dynamic_batching') or {}).get('inf_s'),
 'gb32', (dp.get('resnet50_gb32') or {}).get('img_s'), 'vit', (dp.get('vit_b16_fp8_gb64') or {}).get('img_s'),
 'bs4', (sh.get('resnet50_bs4') or {}).get('img_s_in_flight'), 'vit8', (sh.get('vit_b16_fp8_bs8') or {}).get('img_s_in_flight'),
 'bert1', (c.get('bert_base_bs16') or {}).get('seq_s_1ctx'), 'bert4', (c.get('bert_base_bs16') or {}).get('seq_s_4ctx'),
 'lm_http', (c.get('awd_lstm_get_inference_http') or {}).get('concurrent_req_s'))" | tee -a $OUT/summary.txt
  done
done
