#!/bin/bash
# r4: low-load spin waits in the request executor (HIPZAP_EXEC_SPIN_US, 0 = the sleep-only
# round-3 behaviour): served headline + single-stream latency, interleaved, 3 repetitions
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_s12; mkdir -p $O
B="--steps 300 --warmup 30 --cold-trials 0 --cold-runs 0 --http-clients 0 --dp-figures 0 --dyn-batch 0 --bert-cold 0 --lm-cold 0"
for rep in 1 2 3; do
  for sp in 300 0; do
    HIPZAP_EXEC_SPIN_US=$sp timeout -k 10 200 python bench.py $B > $O/bench_spin${sp}_$rep.json 2> $O/bench_err.log || { tail -20 $O/bench_err.log; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/bench_spin${sp}_$rep.json').read().strip().splitlines()[-1]); print('spin=$sp', d['value'], d['served_sustained']['inf_s'], d['latency_ms_p50_single'], d['latency_ms_p99_single'], d['latency_ms_under_load_p50'])"
  done
done
