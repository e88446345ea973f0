#!/bin/bash
# 2-rank rehearsal of bench.py's multi-rank path on ONE GPU (gloo, ranks folded onto cuda:0);
# not a scaling point -- the driver runs the real 1/2/4/8-GPU curve over RCCL.
set -u
export TMPDIR=/tmp HIPZAP_DIST_BACKEND=gloo HIPZAP_SHARE_GPU=1
mkdir -p gpurun_out
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 100 --warmup 10 > gpurun_out/rehearse_dp2.log 2>&1 || { tail -30 gpurun_out/rehearse_dp2.log; exit 1; }
grep '^{' gpurun_out/rehearse_dp2.log > gpurun_out/rehearse_dp2.json && cat gpurun_out/rehearse_dp2.json
