#!/bin/bash
# r5 s43: per-CU operand-staging rate of a GEMM-like stage loop (scripts/native/cu_stage_bw.hip):
# workgroups per CU x waves x KiB per wave per stage x VGPR / LDS-DMA path
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_s43; mkdir -p $O
timeout -k 10 120 ./scripts/native/cu_stage_bw > $O/cu_stage_bw.jsonl 2>&1; rc=$?; echo "rc=$rc"
cat $O/cu_stage_bw.jsonl
