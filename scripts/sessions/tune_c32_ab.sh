#!/bin/bash
# tune for 32 concurrent streams, then interleaved A/B at 32 streams: c32 table vs the c24 table
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/c32 gpurun_out/tuning
timeout -k 10 700 python -u -m hipzap.engine.tune --model resnet50 --batch 1 --concurrent 32 --report gpurun_out/tune_report_c32.json > gpurun_out/tune_c32.log 2>&1 || { tail -20 gpurun_out/tune_c32.log; exit 1; }
T=hipzap/tuning/resnet50_bs1_c32.json
cp $T gpurun_out/tuning/
for rep in 1 2 3; do
  for v in c32 c24; do
    [ $v = c32 ] && cp gpurun_out/tuning/resnet50_bs1_c32.json $T || rm -f $T
    log=gpurun_out/c32/${v}_$rep.log
    timeout -k 10 200 python bench.py --steps 300 --warmup 30 --cold-runs 0 > $log 2>&1 || { tail -5 $log; exit 1; }
    echo "$v rep$rep $(grep -o '"value": [0-9.]*' $log)"
  done
done
