#!/bin/bash
# r4: non-temporal decoder weight loads (HIPZAP_LMB_DEC_PIPE=8x2nt) vs the default ring, LM tests
# on both, interleaved decode bench (1 / 32 / 64 clients), 2 repetitions
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_s19; mkdir -p $O
HIPZAP_LMB_DEC_PIPE=8x2nt timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_lmbatch_gpu.py tests/test_lmlite_gpu.py > $O/pytest_lm_nt.log 2>&1 || { tail -30 $O/pytest_lm_nt.log; exit 1; }
tail -1 $O/pytest_lm_nt.log
for rep in 1 2; do
for v in 8x2nt 8x2; do
  HIPZAP_LMB_DEC_PIPE=$v timeout -k 10 200 python scripts/bench_lm_batch.py --clients 1 32 64 --requests 12 > $O/lm_${v}_$rep.json 2> $O/lm_err.log || { tail -20 $O/lm_err.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/lm_${v}_$rep.json').read().strip().splitlines()[-1]); print('pipe=$v', [(l['clients'], l['us_per_step'], l['p50_ms'], l['req_per_s']) for l in d['load']])"
done
done
