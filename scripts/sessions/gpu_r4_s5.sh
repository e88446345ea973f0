#!/bin/bash
# r4: fused ResNet kernels (stamps, tests, same-box A/B of the served headline) + the AWD-LSTM
# low-load program (tests, lone-request latency with / without it).
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_s5; mkdir -p $O
timeout -k 10 60 ./scripts/native/block_stamps > $O/stamps.jsonl 2>&1 && cat $O/stamps.jsonl || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_gpu.py tests/test_lmbatch_gpu.py tests/test_lmlite_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for lo in 0 1; do
  HIPZAP_LM_LOWLOAD=$lo timeout -k 10 200 python scripts/bench_lm_batch.py --clients 1 32 --requests 12 > $O/lm_lo$lo.json 2> $O/lm_err.log || { tail -20 $O/lm_err.log; exit 1; }
  tail -c 600 $O/lm_lo$lo.json; echo
done
for pipe in 4x5 4x6 8x2 t2 t1; do
  lay=t3h; dp=$pipe; case $pipe in t*) lay=$pipe; dp=8x2;; esac
  HIPZAP_LMB_LAYER=$lay HIPZAP_LMB_DEC_PIPE=$dp timeout -k 10 200 python scripts/bench_lm_batch.py --clients 1 32 --requests 12 > $O/lm_pipe$pipe.json 2> $O/lm_err.log || { tail -20 $O/lm_err.log; exit 1; }
  tail -c 600 $O/lm_pipe$pipe.json; echo
done
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
