#!/bin/bash
# streams-per-GPU sweep of the headline bench on one box (2 interleaved reps)
set -u
mkdir -p gpurun_out/sweep5
for rep in 1 2; do
  for s in ${SWEEP:-8 12 16 24}; do
    log=gpurun_out/sweep5/s${s}_$rep.log
    timeout -k 10 200 python bench.py --streams $s --steps 300 --warmup 30 --cold-runs 0 > $log 2>&1 || { echo "STOP s$s"; tail -5 $log; exit 1; }
    echo "s$s rep$rep $(grep -o '"value": [0-9.]*' $log)"
  done
done
