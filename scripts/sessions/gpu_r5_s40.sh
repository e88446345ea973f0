#!/bin/bash
# r5 s40: latency-vs-CU-time knobs at 29 dispatches (the served rate is bound by 4 queues x the
# per-request chain, with ~20 % CU-time headroom): layer1 bottleneck tiles 4 rows (98 workgroups),
# layer3 seam slice 64; interleaved (a layer4 K-split slice of 32 is refused by the launcher: ck 64 or 128 at C 512)
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5_s40; mkdir -p $O
B="--steps 20 --warmup 5 --cold-trials 0 --cold-runs 0 --http-clients 0 --dp-figures 0 --dyn-batch 0 --bert-cold 0 --lm-cold 0"
for rep in 1 2; do
  for v in base th4 cs64; do
    E=""
    case $v in
      th4) E="HIPZAP_BNECK_TH=4";;
      cs64) E="HIPZAP_SEAM_CS=64,128";;
    esac
    env $E timeout -k 10 240 python3 bench.py $B > $O/bench_${v}_$rep.log 2>&1 || { tail -20 $O/bench_${v}_$rep.log; exit 1; }
    python3 -c "
import json; j=json.loads(open('$O/bench_${v}_$rep.log').read().strip().splitlines()[-1])
print('$v $rep', j['value'], j['served_sustained']['inf_s'], j['latency_ms_p50_single'])"
  done
done
