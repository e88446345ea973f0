#!/bin/bash
# r4: request-stream count sweep with the fused program (the default 24 was chosen in round 2 for
# the 52-kernel program), interleaved, 2 repetitions; + smoke
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_s15; mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
B="--steps 300 --warmup 30 --cold-trials 0 --cold-runs 0 --http-clients 0 --dp-figures 0 --dyn-batch 0 --bert-cold 0 --lm-cold 0"
for rep in 1 2; do
  for s in 16 24 32 48; do
    timeout -k 10 200 python bench.py --streams $s $B > $O/bench_s${s}_$rep.json 2> $O/bench_err.log || { tail -20 $O/bench_err.log; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/bench_s${s}_$rep.json').read().strip().splitlines()[-1]); print('streams=$s', d['value'], d['served_sustained']['inf_s'], d['latency_ms_under_load_p50'], d['latency_ms_under_load_p99'])"
  done
done
