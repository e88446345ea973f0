#!/bin/bash
# full GPU tier + smoke + driver-form bench, then a same-box A/B of the attention workgroup size
# for L = 128 (BERT bs16: 8 waves -> 192 workgroups on 256 CUs; 4 waves -> 384)
set -u
export TMPDIR=/tmp
bash scripts/gpu_r3_s3.sh || exit 1
O=gpurun_out/r3_att_nw; mkdir -p $O
for v in 64 128 64 128; do
  HIPZAP_ATT_NW8_MINL=$v timeout -k 10 300 python -u scripts/bench_models.py bert-base bert-base-fp8 >> $O/b_$v.jsonl 2>> $O/err.log || { tail -5 $O/err.log; exit 1; }
done
for v in 64 128; do echo "NW8_MINL=$v"; cut -c1-120 $O/b_$v.jsonl; done
