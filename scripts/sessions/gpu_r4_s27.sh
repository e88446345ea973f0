#!/bin/bash
# r4: 16 vs 24 request streams, interleaved, 3 repetitions (same throughput in s15 at 2/3 the latency?)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_s27; mkdir -p $O
B="--steps 400 --warmup 40 --cold-trials 0 --cold-runs 0 --http-clients 0 --dp-figures 0 --dyn-batch 0 --bert-cold 0 --lm-cold 0"
for rep in 1 2 3; do
  for s in 16 24; do
    timeout -k 10 200 python bench.py --streams $s $B > $O/bench_s${s}_$rep.json 2> $O/bench_err.log || { tail -20 $O/bench_err.log; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/bench_s${s}_$rep.json').read().strip().splitlines()[-1]); print('streams=$s', d['value'], d['served_sustained']['inf_s'], d['device_pipelined_inf_s'], d['latency_ms_under_load_p50'], d['latency_ms_under_load_p99'])"
  done
done
