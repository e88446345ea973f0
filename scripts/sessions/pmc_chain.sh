#!/bin/bash
# PMC passes over the ResNet-50 bs=1 served chain (16 request streams, default fuse set), each
# pass its own rocprofv3 run within the per-block counter limits; merged per chain position by
# scripts/pmc_chain.py -> gpurun_out/pmc_chain/chain.json (VERDICT r5 next #1a).
set -u
export TMPDIR=/tmp
OUT=gpurun_out/pmc_chain
mkdir -p $OUT
P1="SQ_WAVES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
P2="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P5="TA_BUSY_avr GRBM_GUI_ACTIVE"
P6="TCC_EA0_ATOMIC_sum GRBM_GUI_ACTIVE"
P3="FETCH_SIZE GRBM_GUI_ACTIVE"
P4="WRITE_SIZE GRBM_GUI_ACTIVE"
BENCH="python3 bench.py --streams 16 --steps 4 --warmup 1 --step-requests 4 --cold-trials 0 --cold-runs 0 --dyn-batch 0 --http-clients 0 --dp-figures 0 --sustained-s 0 ${BENCH_EXTRA:-}"
dirs=""
for pass in ${PASSES:-P1 P2 P3 P4}; do
  ctrs=${!pass}
  timeout -s KILL 240 rocprofv3 --pmc $ctrs -d $OUT/$pass -o run --output-format csv -- $BENCH > $OUT/$pass.log 2>&1
  rc=$?
  echo "pmc $pass rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/$pass.log; exit $rc; fi
  dirs="$dirs $OUT/$pass"
done
python3 scripts/pmc_chain.py $OUT/chain.json $dirs > $OUT/chain.txt && cat $OUT/chain.txt
