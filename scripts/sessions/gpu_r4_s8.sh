#!/bin/bash
# r4: pipelined batched-decode scheduler (two programs, host blocks written while the other replay
# runs): LM GPU tests, then the 1 / 32 / 64-client bench with and without the pipeline.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_s8; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_lmbatch_gpu.py tests/test_lmlite_gpu.py tests/test_lm_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
for pl in 1 0; do
  HIPZAP_LM_PIPELINE=$pl timeout -k 10 200 python scripts/bench_lm_batch.py --clients 1 32 64 --requests 12 > $O/lm_pl${pl}_$rep.json 2> $O/lm_err.log || { tail -20 $O/lm_err.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/lm_pl${pl}_$rep.json').read().strip().splitlines()[-1]); print('pipeline=$pl', [(l['clients'], l['us_per_step'], l['p50_ms'], l['req_per_s']) for l in d['load']])"
done
done
