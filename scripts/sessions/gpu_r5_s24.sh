#!/bin/bash
# r5 s24: PMC passes (own runs, --pmc only) over ViT-B/16 fp8 at batch 64: where the attention
# kernel and the MX GEMMs wait
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r5_s24
mkdir -p $OUT
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
P3="FETCH_SIZE"
run() {
  local pass=$1 ctrs=$2
  timeout -s KILL 150 rocprofv3 --pmc $ctrs -d $OUT/vit64_$pass -o run --output-format csv -- python3 scripts/prof_model.py --model vit-b16-fp8 --batch 64 --iters 4 > $OUT/vit64_$pass.log 2>&1
  local rc=$?
  echo "pmc $pass rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/vit64_$pass.log; exit $rc; fi
  python3 scripts/pmc_summary.py $OUT/vit64_$pass $OUT/vit64_$pass.json > /dev/null && rm -rf $OUT/vit64_$pass
}
run P1 "$P1"
run P2 "$P2"
run P3 "$P3"
python3 - <<'PY'
import json
for p in ("P1", "P2", "P3"):
    d = json.load(open(f"gpurun_out/r5_s24/vit64_{p}.json"))
    pk = list(d.values())[0]["per_kernel"] if "per_kernel" not in d else d["per_kernel"]
    for k, v in pk.items():
        if any(s in k for s in ("attention", "gemm_mx", "layernorm")):
            print(p, k[:60], {c: round(x / max(1, v.get("dispatches", 1)), 1) for c, x in v.items()})
PY
