#!/bin/bash
# r4: BERT-base bs16 LayerNorm fold re-measured on the current GEMMs (lean build) + kernel stats
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4_s16; mkdir -p $O
OUT=$O/ab REPS=2 bash scripts/ab_bert_lnfold.sh || exit 1
for v in 0 1; do
  HIPZAP_LN_FOLD=$v timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof$v -o run -- python3 scripts/bench_models.py bert-base > $O/prof$v.log 2>&1 || { tail -20 $O/prof$v.log; exit 1; }
done
find $O -name "*kernel_stats.csv" | head
