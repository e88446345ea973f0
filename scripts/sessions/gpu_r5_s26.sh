#!/bin/bash
# r5 s26: request-stream count with the 29-dispatch program (16 = the round-4 choice), 2 reps
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5_s26; mkdir -p $O
B="--steps 20 --warmup 5 --cold-trials 0 --cold-runs 0 --http-clients 0 --dp-figures 0 --dyn-batch 0 --bert-cold 0 --lm-cold 0"
for rep in 1 2; do
  for s in 12 16 24 32; do
    timeout -k 10 240 python3 bench.py $B --streams $s > $O/bench_s${s}_$rep.log 2>&1 || { tail -20 $O/bench_s${s}_$rep.log; exit 1; }
    python3 -c "
import json,sys; j=json.loads(open('$O/bench_s${s}_$rep.log').read().strip().splitlines()[-1])
print('streams $s rep $rep', j['value'], j['served_sustained']['inf_s'], j.get('latency_ms_p50'), j.get('latency_ms_p99'))"
  done
done
