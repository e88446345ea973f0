#!/bin/bash
# r5 s45: why the persistent 256 x 256 MX tile (cfg 62) takes ~5 us per k-step: LDS and wait
# counters against cfg 24 on the ViT bs64 shapes (one PMC pass per config)
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5_s45; mkdir -p $O
S="SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY"
for c in 24 62; do
  timeout -s KILL 90 rocprofv3 --pmc $S -d $O/c$c -o p --output-format csv -- python3 scripts/bench_mx.py --cfgs $c > $O/c$c.log 2>&1 || { echo "c$c failed"; tail -5 $O/c$c.log; exit 1; }
done
python3 scripts/pmc_summary.py $O/c24 $O/c62 $O/pmc.json > /dev/null
rm -rf $O/c24 $O/c62
python3 - <<PY
import json
d = json.load(open("$O/pmc.json"))
for run, v in d.items():
    for k, c in v["per_kernel"].items():
        n = c.get("dispatches", 0)
        if n < 20 or "gemm_mx" not in k: continue
        print(run, k[:64], n, {x: round(y / n) for x, y in c.items() if x != "dispatches"})
PY
