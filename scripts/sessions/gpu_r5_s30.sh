#!/bin/bash
# r5 s30: where a ViT-B/16 fp8 bs64 forward spends its time now (kernel stats), for the non-GEMM
# share (attention, LayerNorm, patch embedding, copies)
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5_s30; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/vit -o run --output-format csv -- python3 scripts/prof_model.py --model vit-b16-fp8 --batch 64 --iters 20 > $O/vit.log 2>&1 || { tail -5 $O/vit.log; exit 1; }
tail -1 $O/vit.log
f=$(find $O/vit -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total {tot/1e6:.3f} ms over 20 forwards")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
    print(f'{int(r["Calls"]):6d} {float(r["TotalDurationNs"])/1e6:8.3f} {float(r["AverageNs"])/1e3:8.2f} {100*float(r["TotalDurationNs"])/tot:5.1f}  {r["Name"][:110]}')
PY
find $O/vit -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
rm -rf $O/vit
