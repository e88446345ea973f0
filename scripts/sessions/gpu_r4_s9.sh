#!/bin/bash
# r4: 2-rank rehearsal of the driver's multi-GPU launch (torchrun, gloo, both ranks on cuda:0) with
# this round's defaults; not a scaling point.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HIPZAP_DIST_BACKEND=gloo HIPZAP_SHARE_GPU=1
O=gpurun_out/r4_s9; mkdir -p $O
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 100 --warmup 10 > $O/rehearse_dp2.log 2>&1 || { tail -30 $O/rehearse_dp2.log; exit 1; }
grep '^{' $O/rehearse_dp2.log > $O/rehearse_dp2.json && tail -c 1500 $O/rehearse_dp2.json
