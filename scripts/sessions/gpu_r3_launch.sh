#!/bin/bash
# round 3: self-launched 2-rank rehearsal on ONE GPU (gloo, ranks folded onto cuda:0) + the
# 1-GPU headline with the driver's parameters
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r3_launch
HIPZAP_DIST_BACKEND=gloo HIPZAP_SHARE_GPU=1 timeout -k 10 400 python bench.py --gpus 2 --steps 100 --warmup 10 \
  > gpurun_out/r3_launch/self_launch_2.log 2>&1 || { tail -40 gpurun_out/r3_launch/self_launch_2.log; exit 1; }
grep '^{' gpurun_out/r3_launch/self_launch_2.log | cut -c1-600
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3_launch/n1.log 2>&1 || { tail -40 gpurun_out/r3_launch/n1.log; exit 1; }
grep '^{' gpurun_out/r3_launch/n1.log | cut -c1-400
