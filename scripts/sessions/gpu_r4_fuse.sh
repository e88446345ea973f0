#!/bin/bash
# r4: fused stem + layer1 bottleneck kernels (csrc/block.hip): GPU tests, same-box interleaved A/B of
# the served headline (HIPZAP_FUSE=none vs default), one-request rocprof timeline with fusion.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_fuse; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fused_gpu.py \
  tests/test_engine_gpu.py -k "fused or matches_oracle or uint8 or zero_copy or replay" > $O/pytest.log 2>&1 \
  || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
B="--steps 300 --warmup 30 --cold-trials 0 --cold-runs 0 --http-clients 0 --dp-figures 0 --dyn-batch 0 --bert-cold 0"
for rep in 1 2; do
  for v in none stem,bneck; do
    HIPZAP_FUSE=$v timeout -k 10 200 python bench.py $B > $O/bench_${v/,/_}_$rep.json 2> $O/bench_err.log \
      || { tail -20 $O/bench_err.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$O/bench_${v/,/_}_$rep.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['latency_ms_p50_single'], d['single_stream_inf_s'])"
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/s1 -o run -- python3 bench.py --streams 1 --steps 100 --warmup 5 --cold-trials 0 --cold-runs 0 --http-clients 0 --dp-figures 0 --dyn-batch 0 --bert-cold 0 > $O/bench_s1.log 2>&1 || { tail -20 $O/bench_s1.log; exit 1; }
python3 scripts/rocpd_stats.py $O/s1/run_results.db --timeline stem_kernel pool_fc > $O/one_request_timeline.txt
rm -rf $O/s1
tail -4 $O/one_request_timeline.txt
