#!/bin/bash
# r4: one-request LM program (nb_act = -1: row 0's state only) + one-tile last layer at low load:
# LM GPU tests, then the decode bench with / without it (1 / 32 / 64 clients), 2 repetitions
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_s20; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_lmbatch_gpu.py tests/test_lmlite_gpu.py tests/test_lm_gpu.py > $O/pytest_lm.log 2>&1 || { tail -30 $O/pytest_lm.log; exit 1; }
tail -1 $O/pytest_lm.log
for rep in 1 2; do
for v in 1 0; do
  HIPZAP_LM_SOLO=$v timeout -k 10 200 python scripts/bench_lm_batch.py --clients 1 32 64 --requests 12 > $O/lm_solo${v}_$rep.json 2> $O/lm_err.log || { tail -20 $O/lm_err.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/lm_solo${v}_$rep.json').read().strip().splitlines()[-1]); print('solo=$v', d.get('build_ms'), [(l['clients'], l['us_per_step'], l['p50_ms'], l['req_per_s']) for l in d['load']])"
done
done
