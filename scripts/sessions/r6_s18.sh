#!/bin/bash
# r6 session 18: cold start with 1 vs 4 upload reader threads (HIPZAP_UPLOAD_THREADS; plan, .pth
# without torch, native binary, the LM route); the headline with contexts alternating between the
# normal- and high-priority queue sets (HIPZAP_STREAM_KIND=mixed) vs torch's pool.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r6_s18
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_pth_lite_gpu.py tests/test_plan_gpu.py tests/test_lmlite_gpu.py > $OUT/tests.log 2>&1
rc=$?; tail -n 3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
C="python3 bench.py --cold-trials 15 --lm-cold 1 --bert-cold 0 --dyn-batch 0 --http-clients 0 --dp-figures 0 --config-figures 0 --cold-runs 0 --steps 5 --warmup 2 --sustained-s 0"
for rep in 1 2; do
  for t in 1 4; do
    HIPZAP_UPLOAD_THREADS=$t timeout -k 10 400 $C > $OUT/cold_t${t}_$rep.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { tail -n 5 $OUT/cold_t${t}_$rep.log; exit $rc; }
    grep '^{' $OUT/cold_t${t}_$rep.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); f=d['cold_start_fresh_process']
def ph(k, key):
    return ((f.get(k) or {}).get('median_trial_phases_ms') or {}).get(key)
print('threads $t rep $rep', {k: (f[k].get('p50_ms'), f[k].get('hip_init_ms_p50')) for k in ('plan','pth_lite','native','lm') if isinstance(f.get(k), dict)},
      'plan dma', ph('plan','upload_dma_ms'), 'pthlite raw', ph('pth_lite','upload_raw_ms'), 'lm upload', ph('lm','upload_ms'))" | tee -a $OUT/summary.txt
  done
done
B="python3 bench.py --cold-trials 0 --lm-cold 0 --bert-cold 0 --dyn-batch 0 --http-clients 0 --dp-figures 0 --config-figures 0 --cold-runs 0 --steps 20 --warmup 3"
for rep in 1 2; do
  for k in torch mixed; do
    HIPZAP_STREAM_KIND=$k timeout -k 10 300 $B > $OUT/head_${k}_$rep.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { tail -n 5 $OUT/head_${k}_$rep.log; exit $rc; }
    grep '^{' $OUT/head_${k}_$rep.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print('$k rep $rep value', d['value'], 'sustained', (d.get('served_sustained') or {}).get('inf_s'), 'p99', d.get('latency_ms_under_load_p99'))" | tee -a $OUT/summary.txt
  done
done
