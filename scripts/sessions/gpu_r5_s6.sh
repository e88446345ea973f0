#!/bin/bash
# r5 s7 (= s6 after staging the seam's fp32 t2 in LDS): seams + K-split 3x3 convs (kconv) -- correctness, kconv microbench after the staging
# reorder, headline A/B (base / seam / seam+kconv), kernel trace of seam+kconv
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5_s7; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_seam_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 240 python3 scripts/bench_kconv.py > $O/kconv.jsonl 2>&1 || { tail -20 $O/kconv.jsonl; exit 1; }
grep shape $O/kconv.jsonl
B="--steps 20 --warmup 5 --cold-trials 0 --cold-runs 0 --http-clients 0 --dp-figures 0 --dyn-batch 0 --bert-cold 0 --lm-cold 0"
for rep in 1 2; do
  for v in base seam kconv kconv64; do
    case $v in
      base) F=convpool,bneck,bneck2; CK=32,64;;
      seam) F=convpool,bneck,bneck2,seam; CK=32,64;;
      kconv) F=convpool,bneck,bneck2,seam,kconv; CK=32,64;;
      kconv64) F=convpool,bneck,bneck2,seam,kconv; CK=64,128;;
    esac
    HIPZAP_FUSE=$F HIPZAP_KCONV_CK=$CK timeout -k 10 240 python3 bench.py $B > $O/bench_${v}_$rep.log 2>&1 || { tail -20 $O/bench_${v}_$rep.log; exit 1; }
    python3 -c "
import json,sys; j=json.loads(open('$O/bench_${v}_$rep.log').read().strip().splitlines()[-1])
print('$v $rep', j['value'], j['served_sustained']['inf_s'], j['device_pipelined_inf_s'], j['latency_ms_p50_single'], j['single_stream_inf_s'])"
  done
done
B2="--cold-trials 0 --cold-runs 0 --http-clients 0 --dp-figures 0 --dyn-batch 0 --bert-cold 0 --lm-cold 0"
HIPZAP_FUSE=convpool,bneck,bneck2,seam,kconv timeout -k 10 300 rocprofv3 --kernel-trace -d $O/p -o run -- python3 bench.py --steps 2 --warmup 1 $B2 > $O/prof_16.log 2>&1 || { tail -20 $O/prof_16.log; exit 1; }
python3 scripts/rocpd_stats.py $O/p/run_results.db --cutime preprocess pool_fc > $O/cutime_kconv_16.txt
rm -rf $O/p
sed -n 12,40p $O/cutime_kconv_16.txt | cut -c1-70
