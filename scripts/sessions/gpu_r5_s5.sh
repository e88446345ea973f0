#!/bin/bash
# r5 s5: seam (fixed fp32 consumer ring) + K-split 3x3 kernel correctness; 3x3 microbench; headline
# A/B with/without seams; MX library bar; plan cold-start warm-order A/B
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5_s5; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_seam_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 240 python3 scripts/bench_kconv.py > $O/kconv.jsonl 2>&1 || { tail -20 $O/kconv.jsonl; exit 1; }
cat $O/kconv.jsonl
B="--steps 20 --warmup 5 --cold-trials 0 --cold-runs 0 --http-clients 0 --dp-figures 0 --dyn-batch 0 --bert-cold 0 --lm-cold 0"
for rep in 1 2; do
  for v in base seam seam128; do
    case $v in
      base) F=convpool,bneck,bneck2; CS=128,64;;
      seam) F=convpool,bneck,bneck2,seam; CS=128,64;;
      seam128) F=convpool,bneck,bneck2,seam; CS=128,128;;
    esac
    HIPZAP_FUSE=$F HIPZAP_SEAM_CS=$CS timeout -k 10 240 python3 bench.py $B > $O/bench_${v}_$rep.log 2>&1 || { tail -20 $O/bench_${v}_$rep.log; exit 1; }
    python3 -c "
import json,sys; j=json.loads(open('$O/bench_${v}_$rep.log').read().strip().splitlines()[-1])
print('$v $rep', j['value'], j['served_sustained']['inf_s'], j['device_pipelined_inf_s'], j['latency_ms_p50_single'], j['single_stream_inf_s'])"
  done
done
B2="--cold-trials 0 --cold-runs 0 --http-clients 0 --dp-figures 0 --dyn-batch 0 --bert-cold 0 --lm-cold 0"
HIPZAP_FUSE=convpool,bneck,bneck2,seam timeout -k 10 300 rocprofv3 --kernel-trace -d $O/p -o run -- python3 bench.py --steps 2 --warmup 1 $B2 > $O/prof_16.log 2>&1 || { tail -20 $O/prof_16.log; exit 1; }
python3 scripts/rocpd_stats.py $O/p/run_results.db --cutime preprocess pool_fc > $O/cutime_seam_16.txt
rm -rf $O/p
sed -n 12,40p $O/cutime_seam_16.txt | cut -c1-60
timeout -k 10 180 python3 scripts/bench_mx.py --torch > $O/mx_torch.jsonl 2> $O/mx_torch.err || tail -5 $O/mx_torch.err
timeout -k 10 180 python3 scripts/bench_mx.py --cfgs 24 > $O/mx_cfg24.jsonl 2>&1 || tail -5 $O/mx_cfg24.jsonl
cut -c1-300 $O/mx_torch.jsonl
timeout -k 10 300 python3 scripts/cold_order_ab.py --trials 10 > $O/cold_order_ab.jsonl 2>&1 || tail -5 $O/cold_order_ab.jsonl
tail -1 $O/cold_order_ab.jsonl
