#!/bin/bash
# r5 s36: HIP / HSA runtime switches on the served ResNet-50 bs=1 path (kernel arguments in device
# memory, polled completion signals), interleaved against the default
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5_s36; mkdir -p $O
B="--steps 20 --warmup 5 --cold-trials 0 --cold-runs 0 --http-clients 0 --dp-figures 0 --dyn-batch 0 --bert-cold 0 --lm-cold 0"
for rep in 1 2; do
  for v in base kernarg nointr; do
    E=""
    case $v in
      kernarg) E="HIP_FORCE_DEV_KERNARG=1";;
      nointr) E="HSA_ENABLE_INTERRUPT=0";;
    esac
    env $E timeout -k 10 240 python3 bench.py $B > $O/bench_${v}_$rep.log 2>&1 || { tail -20 $O/bench_${v}_$rep.log; exit 1; }
    python3 -c "
import json; j=json.loads(open('$O/bench_${v}_$rep.log').read().strip().splitlines()[-1])
print('$v $rep', j['value'], j['served_sustained']['inf_s'], j['latency_ms_p50_single'], j['single_stream_inf_s'])"
  done
done
