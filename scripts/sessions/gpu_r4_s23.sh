#!/bin/bash
# r4: LM decoder with 4 vocabulary tiles per wave (HIPZAP_LMB_DEC_TW=4: half the LDS state reads
# per tile) vs 2: LM tests on both, decode bench 1 / 32 / 64 clients, 2 repetitions interleaved
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_s23; mkdir -p $O
for tw in 4 2; do
  HIPZAP_LMB_DEC_TW=$tw timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_lmbatch_gpu.py tests/test_lmlite_gpu.py > $O/pytest_lm_tw$tw.log 2>&1 || { tail -30 $O/pytest_lm_tw$tw.log; exit 1; }
  echo "tw=$tw $(tail -1 $O/pytest_lm_tw$tw.log)"
done
for rep in 1 2; do
for tw in 4 2; do
  HIPZAP_LMB_DEC_TW=$tw timeout -k 10 200 python scripts/bench_lm_batch.py --clients 1 32 64 --requests 12 > $O/lm_tw${tw}_$rep.json 2> $O/lm_err.log || { tail -20 $O/lm_err.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/lm_tw${tw}_$rep.json').read().strip().splitlines()[-1]); print('tw=$tw rep$rep', [(l['clients'], l['us_per_step'], l['p50_ms'], l['req_per_s']) for l in d['load']])"
done
done
