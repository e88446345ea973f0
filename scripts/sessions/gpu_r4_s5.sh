#!/bin/bash
# r4: same-box A/B of the served headline over the fusion kinds (layer1 + layer2 bottlenecks),
# the AWD-LSTM batched decode variants (low-load program, decoder weight ring, layer shapes), then
# the LM GPU tests.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_s5; mkdir -p $O
B="--steps 300 --warmup 30 --cold-trials 0 --cold-runs 0 --http-clients 0 --dp-figures 0 --dyn-batch 0 --bert-cold 0 --lm-cold 0"
for rep in 1 2; do
  for v in none convpool,bneck convpool,bneck,bneck2 convpool,bneck,bneck2:out; do
    f=${v%%:*}; zc=all; [ "$v" != "$f" ] && zc=${v##*:}
    tag=${v//[,:]/_}
    HIPZAP_FUSE=$f HIPZAP_ZERO_COPY=$zc timeout -k 10 200 python bench.py $B > $O/bench_${tag}_$rep.json 2> $O/bench_err.log \
      || { tail -20 $O/bench_err.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$O/bench_${tag}_$rep.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['served_sustained']['inf_s'], d['device_pipelined_inf_s'], d['latency_ms_p50_single'], d['single_stream_inf_s'])"
  done
done
for v in lo0 4x5 4x6 8x2 t2 t1; do
  lo=1; lay=t3h; dp=8x2
  case $v in lo0) lo=0;; t*) lay=$v;; *) dp=$v;; esac
  HIPZAP_LM_LOWLOAD=$lo HIPZAP_LMB_LAYER=$lay HIPZAP_LMB_DEC_PIPE=$dp timeout -k 10 200 python scripts/bench_lm_batch.py --clients 1 32 --requests 12 > $O/lm_$v.json 2> $O/lm_err.log || { tail -20 $O/lm_err.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/lm_$v.json').read().strip().splitlines()[-1]); print('$v', [(l['clients'], l['us_per_step'], l['p50_ms'], l['req_per_s']) for l in d['load']])"
done
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_lmbatch_gpu.py tests/test_lmlite_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
