#!/bin/bash
# r6 session 27: L2 (TCC) counters of the ResNet-50 bs=1 chain on a single-stream replay loop
# (the bench process crashed rocprofv3's TCC passes); one pass, killed hard at 90 s.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r6_s27
mkdir -p $OUT
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES -d $OUT/tcc -o run --output-format csv -- python3 scripts/pmc_resnet_single.py 200 > $OUT/tcc.log 2>&1
rc=$?; echo "tcc pass rc=$rc"; tail -n 3 $OUT/tcc.log; [ $rc -eq 0 ] || exit $rc
python3 scripts/pmc_summary.py $OUT/tcc $OUT/tcc.json > /dev/null && rm -rf $OUT/tcc
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r6_s27/tcc.json"))
for run in d.values():
    rows = []
    for k, v in run["per_kernel"].items():
        h, m, n = v.get("TCC_HIT_sum", 0), v.get("TCC_MISS_sum", 0), max(1, v.get("dispatches", 1))
        rows.append((k[:70], round(h / max(1, h + m), 3), round(v.get("TCC_EA0_RDREQ_sum", 0) / n), round((h + m) / n), n))
    for r in sorted(rows, key=lambda r: -r[3]):
        print(f"{r[0]:70s} hit {r[1]:.3f}  EA rdreq/dispatch {r[2]:>8d}  L2 req/dispatch {r[3]:>8d}  dispatches {r[4]}")
PY
