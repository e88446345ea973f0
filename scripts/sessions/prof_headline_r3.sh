#!/bin/bash
# round-3 final rocprofv3 kernel traces of the headline bench (24 request streams: stats; one
# stream: per-request dispatch timeline). Summaries on the CPU: scripts/rocpd_stats.py.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3_prof; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/s24 -o run -- python3 bench.py --steps 50 --warmup 5 --cold-trials 0 --cold-runs 0 --http-clients 0 --dp-figures 0 --dyn-batch 0 > $O/bench_s24.log 2>&1 || { tail -20 $O/bench_s24.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/s1 -o run -- python3 bench.py --streams 1 --steps 100 --warmup 5 --cold-trials 0 --cold-runs 0 --http-clients 0 --dp-figures 0 --dyn-batch 0 > $O/bench_s1.log 2>&1 || { tail -20 $O/bench_s1.log; exit 1; }

python3 scripts/rocpd_stats.py $O/s24/run_results.db 40 > $O/kernel_stats_24_streams.txt
python3 scripts/rocpd_stats.py $O/s1/run_results.db --timeline preprocess pool_fc > $O/one_request_timeline.txt
rm -rf $O/s24 $O/s1
tail -3 $O/one_request_timeline.txt; head -12 $O/kernel_stats_24_streams.txt
