#!/bin/bash
# r6 session 19: rocprofv3 kernel trace of the final served program (16 request streams, default
# fuse set, deterministic accumulators) -> per-kernel stats and the per-position CU-time table.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r6_s19
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace -d $OUT/prof -o run -- python3 bench.py --cold-trials 0 --lm-cold 0 --bert-cold 0 --dyn-batch 0 --http-clients 0 --dp-figures 0 --config-figures 0 --cold-runs 0 --steps 10 --warmup 3 --sustained-s 0 > $OUT/rocprof.log 2>&1
rc=$?; grep '^{' $OUT/rocprof.log | cut -c1-200; [ $rc -eq 0 ] || { tail -n 20 $OUT/rocprof.log; exit $rc; }
db=$(find $OUT/prof -name '*results.db' | head -n 1)
python3 scripts/rocpd_stats.py "$db" 40 > $OUT/kernel_stats.txt && python3 scripts/rocpd_stats.py "$db" --cutime preprocess pool_fc > $OUT/cutime_final_16_streams.txt
rc=$?; head -n 40 $OUT/cutime_final_16_streams.txt; rm -rf $OUT/prof; exit $rc
