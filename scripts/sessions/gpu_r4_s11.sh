#!/bin/bash
# r4: (1) whole-stem fusion (zero-copy uint8 read inside the conv) vs the default convpool, now
# with every v3 kernel: served + single-stream latency; (2) MALL residency of the LM weight stream
# (EA read requests that go to DRAM vs all EA read requests).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4_s11; mkdir -p $O
B="--steps 300 --warmup 30 --cold-trials 0 --cold-runs 0 --http-clients 0 --dp-figures 0 --dyn-batch 0 --bert-cold 0 --lm-cold 0"
for rep in 1 2 3; do
  for v in convpool,bneck,bneck2 stem,bneck,bneck2; do
    tag=${v//,/_}
    HIPZAP_FUSE=$v timeout -k 10 200 python bench.py $B > $O/bench_${tag}_$rep.json 2> $O/bench_err.log || { tail -20 $O/bench_err.log; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/bench_${tag}_$rep.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['served_sustained']['inf_s'], d['latency_ms_p50_single'], d['single_stream_inf_s'])"
  done
done
P2="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $P2 -d $O/P2 -o run --output-format csv -- python3 scripts/bench_lm_batch.py --clients 32 --requests 2 > $O/P2.log 2>&1
rc=$?; echo "pmc P2 rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/P2.log; exit $rc; }
python3 scripts/pmc_summary.py $O/P2 $O/P2.json > /dev/null && rm -rf $O/P2
python3 -c "
import json; d=json.load(open('$O/P2.json'))['P2']['per_kernel']
for k,v in d.items():
    if 'lmb' in k: print(k[:70], {c: v[c] for c in v}, 'dram/ea=%.3f' % (v.get('TCC_EA0_RDREQ_DRAM_sum',0)/max(1,v.get('TCC_EA0_RDREQ_sum',1))))
"
# (3) would split-K help the BERT bs16 projections? Each split-K-s GEMM (M, N, K) runs like one GEMM
# (s*M, N, K/s) -- same workgroups, same bytes per workgroup -- plus a reduction
timeout -k 10 300 python3 scripts/bench_gemm.py --shapes "2048,768,3072;4096,768,1536;6144,768,1024;8192,768,768;2048,768,768;4096,768,384;6144,768,256;2048,2304,768;4096,2304,384;6144,2304,256;2048,3072,768;4096,3072,384;6144,3072,256" > $O/gemm_splitk.jsonl 2>&1 || { tail -5 $O/gemm_splitk.jsonl; exit 1; }
python3 -c "
import json
for l in open('$O/gemm_splitk.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print(d['M'], d['N'], d['K'], d['hipzap_us'], d['hipzap_cfg'], d['hipblaslt_us'])
"
