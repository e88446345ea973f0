#!/bin/bash
# PMC passes over the fp8 transformer paths (ViT-B/16 fp8 bs64, BERT-base fp8 bs16), one
# rocprofv3 --pmc run per pass (per-block counter limits), summaries -> gpurun_out/pmc8/
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmc8}
mkdir -p $OUT
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F8 SQ_INSTS_MFMA GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F8"
run() {
  local w=$1 pass=$2 ctrs=$3; shift 4
  timeout -s KILL 150 rocprofv3 --pmc $ctrs -d $OUT/${w}_$pass -o run --output-format csv -- "$@" > $OUT/${w}_$pass.log 2>&1
  local rc=$?
  echo "pmc $w $pass rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/${w}_$pass.log; exit $rc; fi
  python3 scripts/pmc_summary.py $OUT/${w}_$pass $OUT/${w}_$pass.json > /dev/null && rm -rf $OUT/${w}_$pass
}
for pass in P1 P2; do
  ctrs=${!pass}
  run vit64fp8 $pass "$ctrs" -- python3 scripts/prof_model.py --model vit-b16-fp8 --batch 64 --iters 5
  run bert16fp8 $pass "$ctrs" -- python3 scripts/prof_model.py --model bert-base-fp8 --batch 16 --iters 10
done
echo done
