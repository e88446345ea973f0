#!/bin/bash
# r6 session 2: layer2 image-pair kernels (tests + batched A/B), determinism cost A/B (hz_fixq vs
# the -DHZ_NO_FIXQ experiments build), then one full driver-form bench run with every figure.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r6_s2
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_fused_gpu.py tests/test_determinism_gpu.py > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 $OUT/tests.log
[ $rc -le 1 ] || exit $rc
summ() { grep '^{' $1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); dp=d.get('dp_scatter') or {}; w=dp.get('dp_shard_w8') or {}
print(' value', d['value'], 'sustained', (d.get('served_sustained') or {}).get('inf_s'), 'p50_single', d['latency_ms_p50_single'],
      'dyn', (d.get('dynamic_batching') or {}).get('inf_s'), 'gb32', (dp.get('resnet50_gb32') or {}).get('img_s'),
      'vit64', (dp.get('vit_b16_fp8_gb64') or {}).get('img_s'), 'bs4', (w.get('resnet50_bs4') or {}).get('img_s'))"; }
B="python3 bench.py --cold-trials 0 --http-clients 0 --config-figures 0 --cold-runs 0 --steps 20 --warmup 5"
for rep in 1 2; do
  for v in 1 0; do
    HIPZAP_B2_IMG=$v timeout -k 10 240 $B > $OUT/b2img${v}_rep$rep.log 2>&1
    rc=$?; echo "b2img=$v rep=$rep rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/b2img${v}_rep$rep.log; exit $rc; }
    summ $OUT/b2img${v}_rep$rep.log
  done
done
B1="python3 bench.py --cold-trials 0 --dyn-batch 0 --http-clients 0 --dp-figures 0 --config-figures 0 --cold-runs 0 --steps 20 --warmup 5"
for rep in 1 2; do
  for lib in default nofixq; do
    if [ $lib = nofixq ]; then export HIPZAP_LIB=hipzap/_lib/libhipzap_exp.so; else unset HIPZAP_LIB; fi
    timeout -k 10 180 $B1 > $OUT/fixq_${lib}_rep$rep.log 2>&1
    rc=$?; echo "fixq lib=$lib rep=$rep rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/fixq_${lib}_rep$rep.log; exit $rc; }
    summ $OUT/fixq_${lib}_rep$rep.log
  done
done
unset HIPZAP_LIB
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_full.log 2>&1
rc=$?; echo "full bench rc=$rc"; [ $rc -eq 0 ] || { tail -20 $OUT/bench_full.log; exit $rc; }
grep '^{' $OUT/bench_full.log > $OUT/bench_full.json
summ $OUT/bench_full.log
python3 -c "
import json; d=json.load(open('$OUT/bench_full.json')); print(json.dumps(d.get('configs'), indent=1)[:3000]); print('cold', d['cold_start_ms_p50'], d.get('cold_start_narrowing'), d['cold_start_pth_ms_p50'])"
timeout -k 10 300 python3 scripts/diag_lmb_vocab.py 8000 20000 40000 60000 90000 > $OUT/lmb_vocab.log 2>&1
rc=$?; echo "lmb vocab rc=$rc"; grep '^{' $OUT/lmb_vocab.log
