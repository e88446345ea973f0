#!/bin/bash
# PMC passes (rocprofv3 --pmc only, each pass its own run within the per-block counter limits)
# over the served workloads: ResNet-50 bs1 x 8 streams (bench.py), BERT-base bs16 and ViT-B/16
# fp8 bs8 (scripts/prof_model.py). Summaries -> gpurun_out/pmc/<workload>_<pass>.json
set -u
export TMPDIR=/tmp
OUT=gpurun_out/pmc
mkdir -p $OUT
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_MFMA GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F8"
P3="FETCH_SIZE"
P4="WRITE_SIZE"
run() {  # run <workload> <pass> <counters> -- <cmd...>
  local w=$1 pass=$2 ctrs=$3; shift 4
  timeout -s KILL 150 rocprofv3 --pmc $ctrs -d $OUT/${w}_$pass -o run --output-format csv -- "$@" > $OUT/${w}_$pass.log 2>&1
  local rc=$?
  echo "pmc $w $pass rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/${w}_$pass.log; exit $rc; fi
  python3 scripts/pmc_summary.py $OUT/${w}_$pass $OUT/${w}_$pass.json > /dev/null && rm -rf $OUT/${w}_$pass
}
for pass in P1 P2 P3 P4; do
  ctrs=${!pass}
  run resnet50_s8 $pass "$ctrs" -- python3 bench.py --streams 8 --steps 20 --warmup 2 --cold-runs 0
  run bert16 $pass "$ctrs" -- python3 scripts/prof_model.py --model bert-base --batch 16 --iters 10
  run vit8fp8 $pass "$ctrs" -- python3 scripts/prof_model.py --model vit-b16-fp8 --batch 8 --iters 10
done
echo done
