#!/bin/bash
# session 3 re-entry check: GPU tier + smoke + the driver's N=1 bench form
set -u
export TMPDIR=/tmp
bash scripts/gpu_r3_full.sh || exit 1
mkdir -p gpurun_out/r3_s5
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3_s5/bench_n1.log 2>&1 || { tail -30 gpurun_out/r3_s5/bench_n1.log; exit 1; }
tail -1 gpurun_out/r3_s5/bench_n1.log | cut -c1-600
