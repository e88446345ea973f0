#!/bin/bash
# r5 s42: hardware queues per process again at 29 dispatches (round 2 measured 4 -> 8 queues as a
# collapse, 7.0k -> 3.4k inf/s): GPU_MAX_HW_QUEUES 4 / 6 / 8 with the default 16 request streams
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5_s42; mkdir -p $O
B="--steps 20 --warmup 5 --cold-trials 0 --cold-runs 0 --http-clients 0 --dp-figures 0 --dyn-batch 0 --bert-cold 0 --lm-cold 0"
for q in 4 6 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 240 python3 bench.py $B > $O/bench_q$q.log 2>&1 || { tail -20 $O/bench_q$q.log; exit 1; }
  python3 -c "
import json; j=json.loads(open('$O/bench_q$q.log').read().strip().splitlines()[-1])
print('queues $q', j['value'], j['served_sustained']['inf_s'], j['latency_ms_p50_single'])"
done
