#!/bin/bash
# r4: full GPU suite after the executor spin + lean request path, then the single-stream latency
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_s13; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { grep -E "FAILED|ERROR|passed|failed" $O/pytest_gpu.log | tail -30; exit 1; }
tail -1 $O/pytest_gpu.log
B="--steps 300 --warmup 30 --cold-trials 0 --cold-runs 0 --http-clients 0 --dp-figures 0 --dyn-batch 0 --bert-cold 0 --lm-cold 0"
for rep in 1 2; do
  timeout -k 10 200 python bench.py $B > $O/bench_$rep.json 2> $O/bench_err.log || { tail -20 $O/bench_err.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_$rep.json').read().strip().splitlines()[-1]); print(d['value'], d['served_sustained']['inf_s'], d['latency_ms_p50_single'], d['latency_ms_p99_single'])"
done
