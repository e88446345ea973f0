#!/bin/bash
# r6 session 9: the cold-start idle-gap sweep (which gap lets the previous child's teardown finish);
# BERT 4-context seq/s against the process's history (fresh / after a 1-context engine / after
# requests through the executor), each in a fresh process, and bench_models.py twice.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r6_s9
mkdir -p $OUT
timeout -k 10 300 python3 -u scripts/cold_gap_sweep.py > $OUT/cold_gap_sweep.jsonl 2>$OUT/cold_gap_sweep.err
rc=$?; cat $OUT/cold_gap_sweep.jsonl; [ $rc -eq 0 ] || { tail -5 $OUT/cold_gap_sweep.err; exit $rc; }
for rep in 1 2; do
  for m in fresh4 fresh4_infer after1 after1_infer; do
    timeout -k 10 120 python3 -u scripts/diag_bert_iters.py --mode $m >> $OUT/bert_modes.jsonl 2>$OUT/bert_modes.err
    rc=$?; [ $rc -eq 0 ] || { tail -5 $OUT/bert_modes.err; exit $rc; }
  done
done
cat $OUT/bert_modes.jsonl
for rep in 1 2; do
  timeout -k 10 200 python3 scripts/bench_models.py bert-base > $OUT/bert_models_$rep.log 2>&1
  rc=$?; grep '^{' $OUT/bert_models_$rep.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
