#!/bin/bash
# r5 s31: ViT patch embedding as patchify + row-major GEMM (K 768) instead of the 16x16/16
# implicit-GEMM conv over 8-channel pixels (K 2048): tune the new GEMM key, tests, ViT dp figures;
# and the persistent attention kernel (HIPZAP_ATT_PERSIST) A/B on the same figures
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5_s31; mkdir -p $O/tuning
timeout -k 10 300 python3 scripts/tune_patch_embed.py > $O/tune.log 2>&1 || { tail -5 $O/tune.log; exit 1; }
grep -h '"set"' $O/tune.log | python3 -c "
import json, sys
for l in sys.stdin:
    j = json.loads(l); print(j['table'], j['set'], j['dropped'], {k: v['best_us'] for k, v in j['report'].items()})"
cp hipzap/tuning/vit-b16*.json $O/tuning/
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_transformers_gpu.py tests/test_fp8_gpu.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"
grep -E 'FAILED|ERROR|passed|failed' $O/pytest.log | tail -12
[ $rc -le 1 ] || exit 1  # a crash or time limit: nothing more on the GPU
B="--steps 5 --warmup 2 --cold-trials 0 --cold-runs 0 --http-clients 0 --dyn-batch 0 --bert-cold 0 --lm-cold 0"
for rep in 1 2; do
  for ap in 0 1; do
    HIPZAP_ATT_PERSIST=$ap timeout -k 10 300 python3 bench.py $B > $O/bench_${ap}_$rep.log 2>&1 || { tail -20 $O/bench_${ap}_$rep.log; exit 1; }
    python3 -c "
import json; j=json.loads(open('$O/bench_${ap}_$rep.log').read().strip().splitlines()[-1]); d=j['dp_scatter']
print('persist=$ap rep $rep', j['value'], d['vit_b16_fp8_gb64']['img_s'], d['dp_shard_w8']['vit_b16_fp8_bs8']['img_s'], d['resnet50_gb32']['img_s'])"
  done
done
