#!/bin/bash
# Interleaved A/B of scripts/bench_models.py between pre-built trees on ONE box.
#   TREES="ab/A ." MODELS="bert-base vit-b16" REPS=2 bash scripts/ab_models.sh
set -u
OUT=${OUT:-gpurun_out/ab_models}
mkdir -p $OUT
for rep in $(seq 1 ${REPS:-2}); do
  for D in ${TREES:-ab/A .}; do
    X=$(basename $(cd $D && pwd))
    log=$OUT/${X}_$rep.log
    (cd $D && timeout -k 10 600 python scripts/bench_models.py ${MODELS:-bert-base}) > $log 2>&1
    rc=$?
    grep -h '^{' $log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l)
    print('$X rep$rep', d.get('model'), 'ctx', d.get('contexts'), d.get('items_per_s'))"
    if [ $rc -ne 0 ]; then echo "STOP $X rc=$rc"; tail -5 $log; exit $rc; fi
  done
done
