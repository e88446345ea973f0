#!/bin/bash
# PMC passes over the MX GEMM tiles on the ViT bs64 shapes: cfg 24 (128x128, 2 WG/CU) vs cfg 47
# (phased 256x128, 1 WG/CU): L2 hit rate / HBM read requests, TA/TD busy, MFMA busy
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r3_pmc_mxp
mkdir -p $OUT
P1="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA"
P2="TA_BUSY_avr TD_BUSY_avr SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
for pass in P1 P2; do
  ctrs=${!pass}
  timeout -s KILL 100 rocprofv3 --pmc $ctrs -d $OUT/$pass -o run --output-format csv -- python3 scripts/bench_mx.py --cfgs 24,47 > $OUT/$pass.log 2>&1
  rc=$?
  echo "pmc $pass rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/$pass.log; exit $rc; fi
  python3 scripts/pmc_summary.py $OUT/$pass $OUT/$pass.json > /dev/null && rm -rf $OUT/$pass
done
echo done
