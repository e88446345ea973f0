#!/bin/bash
# Same-box interleaved A/B of the BERT-base LayerNorm fold (HIPZAP_LN_FOLD=1 vs 0), bs16, 1 and 4 contexts.
set -u
OUT=${OUT:-gpurun_out/ab_lnfold}
mkdir -p $OUT
for rep in $(seq 1 ${REPS:-2}); do
  for v in 1 0; do
    log=$OUT/fold${v}_$rep.log
    HIPZAP_LN_FOLD=$v timeout -k 10 300 python scripts/bench_models.py bert-base > $log 2>&1
    rc=$?
    echo "fold=$v rep$rep rc=$rc $(grep -h '^{' $log | tr '\n' ' ')"
    if [ $rc -ne 0 ]; then echo "STOP rc=$rc"; tail -5 $log; exit $rc; fi
  done
done
