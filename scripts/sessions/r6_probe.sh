#!/bin/bash
# Round 6 probes: cold-start decomposition (HSA / HIP phases, env narrowing A/B) and kernel traces
# of the batched ResNet-50 programs (bs4 = the DP=8 shard of config 3, bs32 = config 3 on one GPU).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r6_probe
timeout -k 10 200 python3 scripts/cold_decompose.py --trials 12 --out gpurun_out/r6_probe/cold_decompose.json > gpurun_out/r6_probe/cold_decompose.log 2>&1
rc=$?; echo "cold_decompose rc=$rc"; tail -40 gpurun_out/r6_probe/cold_decompose.log
[ $rc -eq 0 ] || exit $rc
for b in 4 32; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r6_probe/tr_bs$b -o run --output-format csv -- python3 scripts/prof_model.py --model resnet50 --batch $b --iters 30 > gpurun_out/r6_probe/tr_bs$b.log 2>&1
  rc=$?; echo "trace bs$b rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  python3 scripts/trace_summary.py gpurun_out/r6_probe/tr_bs$b gpurun_out/r6_probe/sum_bs$b > gpurun_out/r6_probe/sum_bs$b.txt 2>&1
  cat gpurun_out/r6_probe/sum_bs$b.txt | tail -50
  rm -rf gpurun_out/r6_probe/tr_bs$b
done
