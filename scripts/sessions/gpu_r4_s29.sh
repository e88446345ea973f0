#!/bin/bash
# r4: a conv table tuned for 16 concurrent streams (the new bench default loads the 8-stream
# table); A/B at 16 streams, interleaved x 3
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_s29; mkdir -p $O
timeout -k 10 900 python -u -m hipzap.engine.tune --model resnet50 --batch 1 --concurrent 16 --report $O/tune_report_c16.json > $O/tune_c16.log 2>&1 || { tail -20 $O/tune_c16.log; exit 1; }
tail -1 $O/tune_c16.log
cp hipzap/tuning/resnet50_bs1_c16.json $O/
B="--steps 400 --warmup 40 --cold-trials 0 --cold-runs 0 --http-clients 0 --dp-figures 0 --dyn-batch 0 --bert-cold 0 --lm-cold 0"
for rep in 1 2 3; do
  for v in c16 c8; do
    if [ $v = c8 ]; then mv hipzap/tuning/resnet50_bs1_c16.json $O/hold.json; fi
    timeout -k 10 200 python bench.py --streams 16 $B > $O/bench_${v}_$rep.json 2> $O/bench_err.log || { tail -20 $O/bench_err.log; exit 1; }
    if [ $v = c8 ]; then mv $O/hold.json hipzap/tuning/resnet50_bs1_c16.json; fi
    python3 -c "import json; d=json.loads(open('$O/bench_${v}_$rep.json').read().strip().splitlines()[-1]); print('table=$v', d['value'], d['served_sustained']['inf_s'], d['latency_ms_under_load_p50'], d['latency_ms_p50_single'])"
  done
done
