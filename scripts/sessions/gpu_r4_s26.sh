#!/bin/bash
# r4: full GPU suite on the final tree + the LM decode bench once (lean build)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_s26; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { grep -E "FAILED|ERROR|passed|failed" $O/pytest_gpu.log | tail -30; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python scripts/bench_lm_batch.py --clients 1 32 64 --requests 12 > $O/lm.json 2> $O/lm_err.log || { tail -20 $O/lm_err.log; exit 1; }
python3 -c "import json; d=json.loads(open('$O/lm.json').read().strip().splitlines()[-1]); print([(l['clients'], l['us_per_step'], l['p50_ms'], l['req_per_s']) for l in d['load']])"
