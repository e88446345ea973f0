#!/bin/bash
# r6 session 21: the LM engine's deferred capture (test under concurrent load) and the LM / .pth
# cold starts with lazy vs eager capture (HIPZAP_LM_CAPTURE) after the zipfile-free reader.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r6_s21
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_lmlite_gpu.py tests/test_native_lm_gpu.py tests/test_pth_lite_gpu.py tests/test_lmbatch_gpu.py > $OUT/tests.log 2>&1
rc=$?; tail -n 4 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $OUT/tests.log | head -n 20; exit $rc; }
C="python3 bench.py --cold-trials 15 --lm-cold 1 --bert-cold 0 --dyn-batch 0 --http-clients 0 --dp-figures 0 --config-figures 0 --cold-runs 0 --steps 5 --warmup 2 --sustained-s 0"
for rep in 1 2; do
  for m in lazy eager; do
    HIPZAP_LM_CAPTURE=$m timeout -k 10 400 $C > $OUT/cold_$m.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { tail -n 5 $OUT/cold_$m.log; exit $rc; }
    grep '^{' $OUT/cold_$m.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); f=d['cold_start_fresh_process']
lm=f.get('lm') or {}
print('$m rep $rep', {k: (f[k].get('p50_ms'), f[k].get('hip_init_ms_p50')) for k in ('plan','pth_lite','native','lm') if isinstance(f.get(k), dict)}, 'lm phases', json.dumps(lm.get('median_trial_phases_ms'))[:400])" | tee -a $OUT/summary.txt
  done
done
