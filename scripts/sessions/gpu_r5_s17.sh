#!/bin/bash
# r5 s17: s16 with the downsample role re-tiled (64 channels x 16 pixels, K halves over the waves, one load round)
# the headline A/B default (tail) vs + xseam at three slice-width pairs, and a CU-time trace
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5_s17; mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_seam_gpu.py > $O/pytest.log 2>&1
echo "pytest rc=$?"
grep -E 'FAILED|ERROR|passed|failed' $O/pytest.log | tail -15
B="--steps 20 --warmup 5 --cold-trials 0 --cold-runs 0 --http-clients 0 --dp-figures 0 --dyn-batch 0 --bert-cold 0 --lm-cold 0"
for rep in 1 2; do
  for v in dsseam dskconv; do
    F=convpool,bneck,bneck2,seam,kconv,tail,xseam; DSA=kconv
    case $v in
      dsseam) DSA=seam;;
    esac
    HIPZAP_FUSE=$F HIPZAP_XSEAM_DS=$DSA timeout -k 10 240 python3 bench.py $B > $O/bench_${v}_$rep.log 2>&1 || { tail -20 $O/bench_${v}_$rep.log; exit 1; }
    python3 -c "
import json,sys; j=json.loads(open('$O/bench_${v}_$rep.log').read().strip().splitlines()[-1])
print('$v $rep', j['value'], j['served_sustained']['inf_s'], j['device_pipelined_inf_s'], j['latency_ms_p50_single'], j['single_stream_inf_s'])"
  done
done
B2="--cold-trials 0 --cold-runs 0 --http-clients 0 --dp-figures 0 --dyn-batch 0 --bert-cold 0 --lm-cold 0"
HIPZAP_FUSE=convpool,bneck,bneck2,seam,kconv,tail,xseam timeout -k 10 300 rocprofv3 --kernel-trace -d $O/p -o run -- python3 bench.py --steps 2 --warmup 1 $B2 > $O/prof_16.log 2>&1 || { tail -20 $O/prof_16.log; exit 1; }
python3 scripts/rocpd_stats.py $O/p/run_results.db --cutime preprocess pool_fc > $O/cutime_16.txt
rm -rf $O/p
cut -c1-100 $O/cutime_16.txt
