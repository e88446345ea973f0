#!/bin/bash
# r6 session 28: AWD-LSTM kernels with the cell update's bias / cell state and the decoder's bias
# fetched at kernel start (one memory round trip less per launch): bitwise tests, then the lone
# request and 32 / 64 clients against the previous build (HIPZAP_LIB=libhipzap_base.so), interleaved.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r6_s28
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_lmbatch_gpu.py tests/test_lmlite_gpu.py tests/test_native_lm_gpu.py tests/test_lm_gpu.py > $OUT/tests.log 2>&1
rc=$?; tail -n 3 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/tests.log | head -n 20; exit $rc; }
for rep in 1 2 3; do
  for lib in base new; do
    if [ $lib = base ]; then export HIPZAP_LIB=$PWD/hipzap/_lib/libhipzap_base.so; else unset HIPZAP_LIB; fi
    timeout -k 10 300 python3 scripts/bench_lm_batch.py --clients 32 64 --requests 8 > $OUT/lm_$lib.log 2>/dev/null
    rc=$?; [ $rc -eq 0 ] || { tail -n 5 $OUT/lm_$lib.log; exit $rc; }
    python3 -c "
import json; d=json.loads(open('$OUT/lm_$lib.log').read().strip().splitlines()[-1])
print('$lib rep $rep lone_ms', d['single_request_ms'], 'us/step', d['single_us_per_step'], 'load', [(r['clients'], r['req_per_s'], r['us_per_step']) for r in d['load']])" | tee -a $OUT/summary.txt
  done
done
unset HIPZAP_LIB
