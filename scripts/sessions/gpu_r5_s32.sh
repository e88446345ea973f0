#!/bin/bash
# r5 s32: ViT-B/16 fp8 bs64 kernel stats for the three lowerings: default (patchify + GEMM,
# one-shot attention), persistent attention, and the old implicit-GEMM conv patch embedding; then
# the same-box dp figures for default vs conv patch embedding, interleaved
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5_s32; mkdir -p $O
stats() {  # $1 = label, env in the caller
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p_$1 -o run --output-format csv -- python3 scripts/prof_model.py --model vit-b16-fp8 --batch 64 --iters 20 > $O/p_$1.log 2>&1 || { tail -5 $O/p_$1.log; return 1; }
  f=$(find $O/p_$1 -name "*kernel_stats.csv" | head -1)
  cp "$f" $O/kernel_stats_$1.csv
  python3 - "$f" "$1" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows if "rocclr" not in r["Name"] and "at::native" not in r["Name"])
print(f"== {sys.argv[2]}: own kernels {tot/20e3:.1f} us per forward")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:8]:
    if "at::native" in r["Name"]: continue
    print(f'{int(r["Calls"]):6d} {float(r["TotalDurationNs"])/20e3:8.1f} us/fwd {float(r["AverageNs"])/1e3:8.2f} us  {r["Name"][:90]}')
PY
  rm -rf $O/p_$1
}
stats default || exit 1
HIPZAP_ATT_PERSIST=1 stats persist || exit 1
HIPZAP_VIT_PATCH=conv stats conv || exit 1
B="--steps 5 --warmup 2 --cold-trials 0 --cold-runs 0 --http-clients 0 --dyn-batch 0 --bert-cold 0 --lm-cold 0"
for rep in 1 2; do
  for pe in gemm conv; do
    HIPZAP_VIT_PATCH=$pe timeout -k 10 300 python3 bench.py $B > $O/bench_${pe}_$rep.log 2>&1 || { tail -20 $O/bench_${pe}_$rep.log; exit 1; }
    python3 -c "
import json; j=json.loads(open('$O/bench_${pe}_$rep.log').read().strip().splitlines()[-1]); d=j['dp_scatter']
print('patch=$pe rep $rep', j['value'], d['vit_b16_fp8_gb64']['img_s'], d['dp_shard_w8']['vit_b16_fp8_bs8']['img_s'], d['resnet50_gb32']['img_s'])"
  done
done
