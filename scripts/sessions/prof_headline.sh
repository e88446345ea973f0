#!/bin/bash
# rocprofv3 kernel traces of the headline bench: 24 request streams (stats) and one stream
# (per-request dispatch timeline). Summaries: scripts/rocpd_stats.py.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_r2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r2/s24 -o run -- python3 bench.py --steps 50 --warmup 5 --cold-trials 0 --cold-runs 0 > gpurun_out/prof_r2/bench_s24.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_r2/s1 -o run -- python3 bench.py --streams 1 --steps 100 --warmup 5 --cold-trials 0 --cold-runs 0 > gpurun_out/prof_r2/bench_s1.log 2>&1
