#!/bin/bash
# r4: (1) 2-rank torchrun rehearsal of the multi-GPU bench path (gloo, both ranks on cuda:0);
# (2) PMC pass over the batched LM decode at 32 rows: L2 hits / misses and memory-side read
# requests per kernel (is the 182 MB weight set served on-die?), plus the counter list.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4_s10; mkdir -p $O
# (0) the projected-embedding first layer: LM tests, then the decode bench with / without it
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_lmbatch_gpu.py tests/test_lmlite_gpu.py > $O/pytest_lm.log 2>&1 || { tail -30 $O/pytest_lm.log; exit 1; }
tail -1 $O/pytest_lm.log
for rep in 1 2; do
for ep in 1 0; do
  HIPZAP_LM_EMBPROJ=$ep timeout -k 10 200 python scripts/bench_lm_batch.py --clients 1 32 64 --requests 12 > $O/lm_ep${ep}_$rep.json 2> $O/lm_err.log || { tail -20 $O/lm_err.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/lm_ep${ep}_$rep.json').read().strip().splitlines()[-1]); print('embproj=$ep', d.get('build_ms'), [(l['clients'], l['us_per_step'], l['p50_ms'], l['req_per_s']) for l in d['load']])"
done
done
timeout -k 10 240 python3 scripts/diag_stream_init.py --trials 5 > $O/stream_init.jsonl 2>&1 || { tail -5 $O/stream_init.jsonl; exit 1; }
tail -1 $O/stream_init.jsonl
rocprofv3 -L > $O/counters_avail.txt 2>&1 || true
grep -i -E "mall|_EA0_|TCC_EA|infinity" $O/counters_avail.txt | head -40 > $O/counters_mall.txt || true
P1="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $P1 -d $O/P1 -o run --output-format csv -- python3 scripts/bench_lm_batch.py --clients 32 --requests 2 > $O/P1.log 2>&1
rc=$?; echo "pmc P1 rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/P1.log; exit $rc; }
python3 scripts/pmc_summary.py $O/P1 $O/P1.json > /dev/null && rm -rf $O/P1
python3 -c "
import json; d=json.load(open('$O/P1.json'))['P1']['per_kernel']
for k,v in d.items():
    if 'lmb' in k: print(k[:80], v)
"
HIPZAP_DIST_BACKEND=gloo HIPZAP_SHARE_GPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 100 --warmup 10 > $O/rehearse_dp2.log 2>&1 || { tail -30 $O/rehearse_dp2.log; exit 1; }
grep '^{' $O/rehearse_dp2.log > $O/rehearse_dp2.json && tail -c 1200 $O/rehearse_dp2.json
# (3) request input through the SDMA engines instead of a zero-copy PCIe read inside the
# preprocess kernel (which holds a compute-queue slot for the whole transfer): same-box A/B
B="--steps 300 --warmup 30 --cold-trials 0 --cold-runs 0 --http-clients 0 --dp-figures 0 --dyn-batch 0 --bert-cold 0 --lm-cold 0"
for rep in 1 2; do
  for v in all:0 out:0 out:1 all:1; do
    zc=${v%%:*}; sd=${v##*:}
    HSA_ENABLE_SDMA=$sd HIPZAP_KEEP_SDMA=$sd HIPZAP_ZERO_COPY=$zc timeout -k 10 200 python bench.py $B > $O/bench_${zc}_sdma${sd}_$rep.json 2> $O/bench_err.log || { tail -20 $O/bench_err.log; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/bench_${zc}_sdma${sd}_$rep.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['served_sustained']['inf_s'], d['latency_ms_p50_single'])"
  done
done
