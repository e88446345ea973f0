#!/bin/bash
# r5 s19: where ViT-B/16 fp8 at batch 64 spends its time (kernel stats), and the smoke entry point
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5_s19; mkdir -p $O
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; echo "smoke rc=$?"; tail -2 $O/smoke.log
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/pv -o run -- python3 scripts/prof_model.py --model vit-b16-fp8 --batch 64 --iters 10 > $O/prof_vit.log 2>&1 || { tail -20 $O/prof_vit.log; exit 1; }
db=$(find $O/pv -name '*results.db' | head -1)
python3 scripts/rocpd_stats.py "$db" 16 > $O/kernel_stats_vit_fp8_bs64.txt
rm -rf $O/pv
cut -c1-170 $O/kernel_stats_vit_fp8_bs64.txt
