#!/bin/bash
# r5 s2: seam kernel correctness, then an interleaved A/B of the served headline with / without
# seams and the slice-width variants
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5_s2; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_seam_gpu.py tests/test_fused_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
B="--steps 300 --warmup 20 --cold-trials 0 --cold-runs 0 --http-clients 0 --dp-figures 0 --dyn-batch 0 --bert-cold 0 --lm-cold 0"
for rep in 1 2; do
  for v in base seam seam64 seam128; do
    case $v in
      base) F=convpool,bneck,bneck2; CS=128,64;;
      seam) F=convpool,bneck,bneck2,seam; CS=128,64;;
      seam64) F=convpool,bneck,bneck2,seam; CS=64,64;;
      seam128) F=convpool,bneck,bneck2,seam; CS=128,128;;
    esac
    HIPZAP_FUSE=$F HIPZAP_SEAM_CS=$CS timeout -k 10 240 python3 bench.py $B > $O/bench_${v}_$rep.log 2>&1 || { tail -20 $O/bench_${v}_$rep.log; exit 1; }
    python3 -c "
import json,sys; j=json.loads(open('$O/bench_${v}_$rep.log').read().strip().splitlines()[-1])
print('$v $rep', j['value'], j['served_sustained']['inf_s'], j['device_pipelined_inf_s'], j['latency_ms_p50_single'], j['single_stream_inf_s'])"
  done
done
