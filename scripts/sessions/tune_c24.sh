#!/bin/bash
# tune ResNet-50 bs1 launch configs for 24 concurrent request streams, then bench 24 streams with it
set -u
mkdir -p gpurun_out/tuning gpurun_out/c24
timeout -k 10 700 python -u -m hipzap.engine.tune --model resnet50 --batch 1 --concurrent 24 --report gpurun_out/tune_report_c24.json > gpurun_out/tune_c24.log 2>&1 || { tail -20 gpurun_out/tune_c24.log; exit 1; }
cp hipzap/tuning/resnet50_bs1_c24.json gpurun_out/tuning/
for rep in 1 2; do
  for s in 24 32; do
    log=gpurun_out/c24/s${s}_$rep.log
    timeout -k 10 200 python bench.py --streams $s --steps 300 --warmup 30 --cold-runs 0 > $log 2>&1 || { tail -5 $log; exit 1; }
    echo "s$s rep$rep $(grep -o '"value": [0-9.]*' $log)"
  done
done
