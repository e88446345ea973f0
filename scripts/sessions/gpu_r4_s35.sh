#!/bin/bash
# r4 (for round 5): PMC passes over the MX GEMM on the ViT bs64 shapes, cfg 24 vs the ping-pong
# cfg 34 / 35 (experiments build): MFMA busy, LDS bank conflicts, wait cycles, TA/TD busy
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
export HIPZAP_LIB=$PWD/hipzap/_lib/libhipzap_exp.so
OUT=gpurun_out/r4_pmc_mxpp
mkdir -p $OUT
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F8 SQ_INSTS_MFMA GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F8"
P3="TA_BUSY_avr TD_BUSY_avr SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
for pass in P1 P2 P3; do
  ctrs=${!pass}
  timeout -s KILL 100 rocprofv3 --pmc $ctrs -d $OUT/$pass -o run --output-format csv -- python3 scripts/bench_mx.py --cfgs 24,34,35 > $OUT/$pass.log 2>&1
  rc=$?
  echo "pmc $pass rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/$pass.log; exit $rc; fi
  python3 scripts/pmc_summary.py $OUT/$pass $OUT/$pass.json > /dev/null && rm -rf $OUT/$pass
done
echo done
