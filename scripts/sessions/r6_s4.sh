#!/bin/bash
# r6 session 4: native GET /inference test, BERT 1/4-context and LM engine-level reference figures
# (scripts/bench_models.py, scripts/bench_lm_batch.py) next to scripts/bench_configs.py.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r6_s4
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_native_lm_gpu.py > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python3 scripts/bench_models.py bert-base > $OUT/bench_models_bert.log 2>&1
rc=$?; echo "bench_models rc=$rc"; grep '^{' $OUT/bench_models_bert.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/bench_lm_batch.py --clients 1 32 64 --requests 10 > $OUT/bench_lm_batch.log 2>&1
rc=$?; echo "bench_lm_batch rc=$rc"; grep '^{' $OUT/bench_lm_batch.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/bench_configs.py --device 0 > $OUT/configs.log 2>&1
rc=$?; echo "configs rc=$rc"; grep '^{' $OUT/configs.log | cut -c1-3000
timeout -k 10 200 python3 scripts/cold_decompose.py --trials 10 --out $OUT/cold_decompose.json > $OUT/cold_decompose.log 2>&1; echo "cold_decompose rc=$?"; python3 -c "import json; d=json.load(open(\"$OUT/cold_decompose.json\")); [print(a, m) for a, m in d[\"median\"].items()]"
