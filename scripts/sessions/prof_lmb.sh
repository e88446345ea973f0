#!/bin/bash
# rocprofv3 kernel trace of the batched AWD-LSTM decode under 32 concurrent 200-word requests
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_lmb
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_lmb/c32 -o run -- python3 scripts/bench_lm_batch.py --clients 32 --requests 4 > gpurun_out/prof_lmb/bench.log 2>&1 || { tail -30 gpurun_out/prof_lmb/bench.log; exit 1; }
db=$(find gpurun_out/prof_lmb/c32 -name '*results.db' | head -1)
python3 scripts/rocpd_stats.py "$db" 20 > gpurun_out/prof_lmb/kernel_stats.txt
python3 scripts/rocpd_stats.py "$db" --timeline lmb_layer_kernelILi2ELb1 lmb_dec_kernel > gpurun_out/prof_lmb/one_step.txt
cat gpurun_out/prof_lmb/kernel_stats.txt gpurun_out/prof_lmb/one_step.txt
