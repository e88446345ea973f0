#!/bin/bash
# r6 session 3: tests of the auto image-pair rule, the config figures in a fresh child, the bs4
# K-split slice A/B (HIPZAP_KCONV_CK), then the full driver-form bench.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r6_s3
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_fused_gpu.py tests/test_native_lm_gpu.py -k "two_images or native" > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 scripts/bench_configs.py --device 0 > $OUT/configs.log 2>&1
rc=$?; echo "configs rc=$rc"; grep '^{' $OUT/configs.log | cut -c1-1500
[ $rc -eq 0 ] || exit $rc
summ() { grep '^{' $1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); dp=d.get('dp_scatter') or {}; w=dp.get('dp_shard_w8') or {}
print(' value', d['value'], 'sustained', (d.get('served_sustained') or {}).get('inf_s'), 'p50_single', d['latency_ms_p50_single'],
      'dyn', (d.get('dynamic_batching') or {}).get('inf_s'), 'gb32', (dp.get('resnet50_gb32') or {}).get('img_s'),
      'bs4', (w.get('resnet50_bs4') or {}).get('img_s'))"; }
B="python3 bench.py --cold-trials 0 --http-clients 0 --config-figures 0 --cold-runs 0 --dyn-batch 0 --steps 20 --warmup 5"
for rep in 1 2; do
  for ck in 32,64 64,128; do
    HIPZAP_KCONV_CK=$ck timeout -k 10 240 $B > $OUT/ck${ck/,/_}_rep$rep.log 2>&1
    rc=$?; echo "ck=$ck rep=$rep rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/ck${ck/,/_}_rep$rep.log; exit $rc; }
    summ $OUT/ck${ck/,/_}_rep$rep.log
  done
done
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_full.log 2>&1
rc=$?; echo "full bench rc=$rc"; [ $rc -eq 0 ] || { tail -20 $OUT/bench_full.log; exit $rc; }
grep '^{' $OUT/bench_full.log > $OUT/bench_full.json
summ $OUT/bench_full.log
python3 -c "
import json; d=json.load(open('$OUT/bench_full.json')); c=d.get('configs') or {}
print(json.dumps({k: {kk: vv for kk, vv in (v or {}).items() if 'ms' in kk or '_s' in kk} for k, v in c.items()}))
print('cold', d['cold_start_ms_p50'], d.get('cold_start_narrowing'), 'pth', d['cold_start_pth_ms_p50'], 'native', d['cold_start_native_ms_p50'], 'lm', d['cold_start_lm_ms_p50'])
print('own', {k: (v or {}).get('own_ms_p50') for k, v in d['cold_start_fresh_process'].items() if isinstance(v, dict)})"
