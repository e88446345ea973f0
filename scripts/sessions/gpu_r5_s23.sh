#!/bin/bash
# r5 s23: CU-time trims under 16 streams: layer4 K-split slice 128 (64 workgroups instead of 128),
# with and without the layer3 downsample seam; 3 interleaved reps
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5_s23; mkdir -p $O
B="--steps 20 --warmup 5 --cold-trials 0 --cold-runs 0 --http-clients 0 --dp-figures 0 --dyn-batch 0 --bert-cold 0 --lm-cold 0"
for rep in 1 2 3; do
  for v in base ck128 ck128ds; do
    F=convpool,bneck,bneck2,seam,kconv,tail,xseam; CK=32,64
    case $v in
      ck128) CK=32,128;;
      ck128ds) CK=32,128; F=$F,dsseam;;
    esac
    HIPZAP_FUSE=$F HIPZAP_KCONV_CK=$CK timeout -k 10 240 python3 bench.py $B > $O/bench_${v}_$rep.log 2>&1 || { tail -20 $O/bench_${v}_$rep.log; exit 1; }
    python3 -c "
import json,sys; j=json.loads(open('$O/bench_${v}_$rep.log').read().strip().splitlines()[-1])
print('$v $rep', j['value'], j['served_sustained']['inf_s'], j['device_pipelined_inf_s'], j['latency_ms_p50_single'], j['single_stream_inf_s'])"
  done
done
