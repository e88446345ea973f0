#!/bin/bash
# r5 s8: kconv at every layer3/layer4 3x3 (the stride-2 first blocks included, preset by the pair),
# seams stage t2 in LDS -- correctness, headline A/B, slice-width variants, kernel trace
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5_s8; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_seam_gpu.py tests/test_fused_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
B="--steps 20 --warmup 5 --cold-trials 0 --cold-runs 0 --http-clients 0 --dp-figures 0 --dyn-batch 0 --bert-cold 0 --lm-cold 0"
for rep in 1 2; do
  for v in base kconv kconv_cs128 kconv_cs64; do
    F=convpool,bneck,bneck2,seam,kconv; CS=128,64
    case $v in
      base) F=convpool,bneck,bneck2;;
      kconv_cs128) CS=128,128;;
      kconv_cs64) CS=64,64;;
    esac
    HIPZAP_FUSE=$F HIPZAP_SEAM_CS=$CS timeout -k 10 240 python3 bench.py $B > $O/bench_${v}_$rep.log 2>&1 || { tail -20 $O/bench_${v}_$rep.log; exit 1; }
    python3 -c "
import json,sys; j=json.loads(open('$O/bench_${v}_$rep.log').read().strip().splitlines()[-1])
print('$v $rep', j['value'], j['served_sustained']['inf_s'], j['device_pipelined_inf_s'], j['latency_ms_p50_single'], j['single_stream_inf_s'])"
  done
done
B2="--cold-trials 0 --cold-runs 0 --http-clients 0 --dp-figures 0 --dyn-batch 0 --bert-cold 0 --lm-cold 0"
HIPZAP_FUSE=convpool,bneck,bneck2,seam,kconv timeout -k 10 300 rocprofv3 --kernel-trace -d $O/p -o run -- python3 bench.py --steps 2 --warmup 1 $B2 > $O/prof_16.log 2>&1 || { tail -20 $O/prof_16.log; exit 1; }
python3 scripts/rocpd_stats.py $O/p/run_results.db --cutime preprocess pool_fc > $O/cutime_kconv_16.txt
rm -rf $O/p
HIPZAP_FUSE=convpool,bneck,bneck2,seam,kconv timeout -k 10 300 rocprofv3 --kernel-trace -d $O/p -o run -- python3 bench.py --streams 1 --steps 2 --warmup 1 $B2 > $O/prof_1.log 2>&1 || { tail -20 $O/prof_1.log; exit 1; }
python3 scripts/rocpd_stats.py $O/p/run_results.db --cutime preprocess pool_fc > $O/cutime_kconv_1.txt
rm -rf $O/p
cut -c1-72 $O/cutime_kconv_16.txt
