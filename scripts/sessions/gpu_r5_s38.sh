#!/bin/bash
# r5 s38: ViT attention workgroup size at L = 197 (4 / 8 / 16 waves: HIPZAP_ATT_NW8_MINL=256 forces
# the 4-wave kernel, HIPZAP_ATT_NW16=1 the 16-wave one), interleaved on the config-5 dp figures
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5_s38; mkdir -p $O
B="--steps 5 --warmup 2 --cold-trials 0 --cold-runs 0 --http-clients 0 --dyn-batch 0 --bert-cold 0 --lm-cold 0"
for rep in 1 2; do
  for v in nw8 nw4 nw16; do
    E=""
    case $v in
      nw4) E="HIPZAP_ATT_NW8_MINL=256";;
      nw16) E="HIPZAP_ATT_NW16=1";;
    esac
    env $E timeout -k 10 300 python3 bench.py $B > $O/bench_${v}_$rep.log 2>&1 || { tail -20 $O/bench_${v}_$rep.log; exit 1; }
    python3 -c "
import json; j=json.loads(open('$O/bench_${v}_$rep.log').read().strip().splitlines()[-1]); d=j['dp_scatter']
print('$v rep $rep', d['vit_b16_fp8_gb64']['img_s'], d['dp_shard_w8']['vit_b16_fp8_bs8']['img_s'])"
  done
done
