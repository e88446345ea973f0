#!/bin/bash
# r5 s1: baseline on this round's box -- driver-form bench + rocprofv3 CU-time accounting of the
# headline at the 16-stream default (VERDICT r4 "next round" 1a)
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5_s1; mkdir -p $O
B="--cold-trials 0 --cold-runs 0 --http-clients 0 --dp-figures 0 --dyn-batch 0 --bert-cold 0 --lm-cold 0"
timeout -k 10 300 python3 bench.py --steps 300 --warmup 20 $B > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/s16 -o run -- python3 bench.py --steps 50 --warmup 5 $B > $O/prof_s16.log 2>&1 || { tail -20 $O/prof_s16.log; exit 1; }
python3 scripts/rocpd_stats.py $O/s16/run_results.db 40 > $O/kernel_stats_16_streams.txt
python3 scripts/rocpd_stats.py $O/s16/run_results.db --cutime preprocess pool_fc > $O/cutime_16_streams.txt
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/s1 -o run -- python3 bench.py --streams 1 --steps 100 --warmup 5 $B > $O/prof_s1.log 2>&1 || { tail -20 $O/prof_s1.log; exit 1; }
python3 scripts/rocpd_stats.py $O/s1/run_results.db --cutime preprocess pool_fc > $O/cutime_1_stream.txt
rm -rf $O/s16 $O/s1
cat $O/cutime_16_streams.txt
