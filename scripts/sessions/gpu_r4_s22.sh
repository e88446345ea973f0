#!/bin/bash
# r4: LM decoder OOB slots + layer k-step clamp: LM tests, decode bench 1 / 32 / 64 clients x 2, profile
# to re-read the next workgroup's tiles): LM tests, decode bench 1 / 32 / 64 clients x 2, profile
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4_s22; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_lmbatch_gpu.py tests/test_lmlite_gpu.py tests/test_lm_gpu.py > $O/pytest_lm.log 2>&1 || { tail -30 $O/pytest_lm.log; exit 1; }
tail -1 $O/pytest_lm.log
for rep in 1 2; do
  timeout -k 10 200 python scripts/bench_lm_batch.py --clients 1 32 64 --requests 12 > $O/lm_$rep.json 2> $O/lm_err.log || { tail -20 $O/lm_err.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/lm_$rep.json').read().strip().splitlines()[-1]); print('rep$rep', [(l['clients'], l['us_per_step'], l['p50_ms'], l['req_per_s']) for l in d['load']])"
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/lmc32 -o run -- python3 scripts/bench_lm_batch.py --clients 32 --requests 4 > $O/lmc32.log 2>&1 || { tail -20 $O/lmc32.log; exit 1; }
echo done
