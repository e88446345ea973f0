#!/bin/bash
# r4: the new defaults end to end -- full GPU test suite, smoke, the full bench (cold-start fields
# included), rocprofv3 traces of the headline (24 streams: stats; one stream: per-request timeline)
# and of the batched LM decode at 32 rows.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_s7; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { grep -E "FAILED|ERROR|passed|failed" $O/pytest_gpu.log | tail -40; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench_err.log || { tail -20 $O/bench_err.log; exit 1; }
tail -c 3000 $O/bench.json; echo
B="--cold-trials 0 --cold-runs 0 --http-clients 0 --dp-figures 0 --dyn-batch 0 --bert-cold 0 --lm-cold 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/s24 -o run -- python3 bench.py --steps 50 --warmup 5 $B > $O/bench_s24.log 2>&1 || { tail -20 $O/bench_s24.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/s1 -o run -- python3 bench.py --streams 1 --steps 100 --warmup 5 $B > $O/bench_s1.log 2>&1 || { tail -20 $O/bench_s1.log; exit 1; }
python3 scripts/rocpd_stats.py $O/s24/run_results.db 40 > $O/kernel_stats_24_streams.txt
python3 scripts/rocpd_stats.py $O/s1/run_results.db --timeline preprocess pool_fc > $O/one_request_timeline.txt
rm -rf $O/s24 $O/s1
tail -3 $O/one_request_timeline.txt; head -12 $O/kernel_stats_24_streams.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/lmb -o run -- python3 scripts/bench_lm_batch.py --clients 32 --requests 4 > $O/lmb.log 2>&1 || { tail -20 $O/lmb.log; exit 1; }
db=$(find $O/lmb -name '*results.db' | head -1)
python3 scripts/rocpd_stats.py "$db" 12 > $O/kernel_stats_lmb_c32.txt
rm -rf $O/lmb
cat $O/kernel_stats_lmb_c32.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/lmb1 -o run -- python3 scripts/bench_lm_batch.py --clients 1 --requests 8 > $O/lmb1.log 2>&1 || { tail -20 $O/lmb1.log; exit 1; }
db=$(find $O/lmb1 -name '*results.db' | head -1)
python3 scripts/rocpd_stats.py "$db" 12 > $O/kernel_stats_lmb_c1.txt
python3 scripts/rocpd_stats.py "$db" --timeline lmb_admit lmb_dec_kernel > $O/lmb_c1_timeline.txt
rm -rf $O/lmb1
cat $O/kernel_stats_lmb_c1.txt; tail -12 $O/lmb_c1_timeline.txt
