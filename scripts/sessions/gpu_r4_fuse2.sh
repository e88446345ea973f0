#!/bin/bash
# r4 fused kernels v2 (pipelined LDS operands, biases preloaded): tests, same-box A/B, rocprof
# one-request timeline and 24-stream kernel stats (durations under concurrency).
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_fuse2; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fused_gpu.py > $O/pytest.log 2>&1 \
  || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
B="--steps 300 --warmup 30 --cold-trials 0 --cold-runs 0 --http-clients 0 --dp-figures 0 --dyn-batch 0 --bert-cold 0"
for rep in 1 2; do
  for v in none stem,bneck; do
    HIPZAP_FUSE=$v timeout -k 10 200 python bench.py $B > $O/bench_${v/,/_}_$rep.json 2> $O/bench_err.log \
      || { tail -20 $O/bench_err.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$O/bench_${v/,/_}_$rep.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['served_sustained']['inf_s'], d['latency_ms_p50_single'], d['single_stream_inf_s'])"
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/s1 -o run -- python3 bench.py --streams 1 --steps 100 --warmup 5 --cold-trials 0 --cold-runs 0 --http-clients 0 --dp-figures 0 --dyn-batch 0 --bert-cold 0 > $O/bench_s1.log 2>&1 || { tail -20 $O/bench_s1.log; exit 1; }
python3 scripts/rocpd_stats.py $O/s1/run_results.db --timeline stem_kernel pool_fc > $O/one_request_timeline.txt
rm -rf $O/s1
for v in none stem,bneck; do
  HIPZAP_FUSE=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/s24 -o run -- python3 bench.py --steps 50 --warmup 5 --cold-trials 0 --cold-runs 0 --http-clients 0 --dp-figures 0 --dyn-batch 0 --bert-cold 0 > $O/bench_s24.log 2>&1 || { tail -20 $O/bench_s24.log; exit 1; }
  python3 scripts/rocpd_stats.py $O/s24/run_results.db 40 > $O/kernel_stats_24_streams_${v/,/_}.txt
  rm -rf $O/s24
done
head -12 $O/one_request_timeline.txt; tail -2 $O/one_request_timeline.txt
head -14 $O/kernel_stats_24_streams_stem_bneck.txt
