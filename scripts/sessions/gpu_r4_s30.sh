#!/bin/bash
# r4 final: rocprofv3 kernel stats of the headline at the 16-stream default
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4_s30; mkdir -p $O
B="--cold-trials 0 --cold-runs 0 --http-clients 0 --dp-figures 0 --dyn-batch 0 --bert-cold 0 --lm-cold 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/s16 -o run -- python3 bench.py --steps 50 --warmup 5 $B > $O/bench_s16.log 2>&1 || { tail -20 $O/bench_s16.log; exit 1; }
python3 scripts/rocpd_stats.py $O/s16/run_results.db 40 > $O/kernel_stats_16_streams.txt
rm -rf $O/s16
head -14 $O/kernel_stats_16_streams.txt
