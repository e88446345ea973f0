#!/bin/bash
# r4: in-kernel phase stamps of the fused ResNet kernels (scripts/native/block_stamps.hip, built on
# the CPU host), then the fused-v2 session.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_stamps; mkdir -p $O
timeout -k 10 60 ./scripts/native/block_stamps > $O/stamps.jsonl 2>&1 || { cat $O/stamps.jsonl; exit 1; }
cat $O/stamps.jsonl
bash scripts/sessions/gpu_r4_fuse2.sh
