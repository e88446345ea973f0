#!/bin/bash
# r4: conv+maxpool fusion after the standalone preprocess (convpool) vs the full stem; stamps with
# the conv2 MFMA / epilogue split; same-box interleaved A/B of the served headline.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_fuse4; mkdir -p $O
timeout -k 10 60 ./scripts/native/block_stamps > $O/stamps.jsonl 2>&1 && cat $O/stamps.jsonl
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B="--steps 300 --warmup 30 --cold-trials 0 --cold-runs 0 --http-clients 0 --dp-figures 0 --dyn-batch 0 --bert-cold 0 --lm-cold 0"
for rep in 1 2; do
  for v in none bneck convpool,bneck convpool,bneck:out stem,bneck:out; do
    f=${v%%:*}; zc=all; [ "$v" != "$f" ] && zc=${v##*:}
    tag=${v//[,:]/_}
    HIPZAP_FUSE=$f HIPZAP_ZERO_COPY=$zc timeout -k 10 200 python bench.py $B > $O/bench_${tag}_$rep.json 2> $O/bench_err.log \
      || { tail -20 $O/bench_err.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$O/bench_${tag}_$rep.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['served_sustained']['inf_s'], d['device_pipelined_inf_s'], d['latency_ms_p50_single'], d['single_stream_inf_s'])"
  done
done
