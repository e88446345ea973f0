#!/bin/bash
# r6 session 24: SQ / TA counters of the role-split MX GEMM (cfg 40) against cfg 24 on the ViT-B/16
# gb64 shapes: where the role-split kernel's time goes.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r6_s24
mkdir -p $OUT
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F8 SQ_INSTS_MFMA GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_LDS"
P3="TA_BUSY_avr SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
for pass in P1 P2 P3; do
  ctrs=${!pass}
  timeout -s KILL 100 rocprofv3 --pmc $ctrs -d $OUT/$pass -o run --output-format csv -- python3 scripts/bench_mx.py --cfgs 24,40 > $OUT/$pass.log 2>&1
  rc=$?
  echo "pmc $pass rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 5 $OUT/$pass.log; exit $rc; fi
  python3 scripts/pmc_summary.py $OUT/$pass $OUT/$pass.json > /dev/null && rm -rf $OUT/$pass
done
python3 - <<'PY'
import json
O = "gpurun_out/r6_s24"
tot = {}
for p in ("P1", "P2", "P3"):
    d = json.load(open(f"{O}/{p}.json"))
    for run in d.values():
        for k, v in run["per_kernel"].items():
            if "gemm_mx" not in k:
                continue
            name = "cfg40 role-split" if "rs_kernel" in k else "cfg24"
            t = tot.setdefault(name, {})
            for c, x in v.items():
                t[c] = t.get(c, 0) + x
for name, t in tot.items():
    wc = t.get("SQ_WAVE_CYCLES", 1)
    print(name, {"mfma_busy/cu_busy": round(t.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / max(1, t.get("SQ_BUSY_CU_CYCLES", 1)), 3),
                 "wait_any/wave_cycles": round(t.get("SQ_WAIT_ANY", 0) / wc, 3),
                 "wait_inst_any/wave_cycles": round(t.get("SQ_WAIT_INST_ANY", 0) / wc, 3),
                 "active_inst/wave_cycles": round(t.get("SQ_ACTIVE_INST_ANY", 0) / wc, 3),
                 "lds_wait/wave_cycles": round(t.get("SQ_WAIT_INST_LDS", 0) / wc, 3),
                 "lds_bank_conflict/lds_active": round(t.get("SQ_LDS_BANK_CONFLICT", 0) / max(1, t.get("SQ_LDS_IDX_ACTIVE", 1)), 4),
                 "busy_cycles": t.get("SQ_BUSY_CYCLES"), "waves": t.get("SQ_WAVES"), "ta_busy_avr": t.get("TA_BUSY_avr")})
PY
