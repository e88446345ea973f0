#!/bin/bash
# Sweep HIP hardware queues x concurrent request streams for the headline bench (1 GPU).
set -u
mkdir -p gpurun_out/sweep
for q in ${QUEUES:-4 8 16}; do
  for s in ${STREAMS:-8 16}; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --streams $s --steps 300 --warmup 30 --cold-runs 0 \
      > gpurun_out/sweep/q${q}_s${s}.log 2>&1
    rc=$?
    echo "q=$q s=$s rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/sweep/q${q}_s${s}.log)"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  done
done
