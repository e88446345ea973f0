#!/bin/bash
# PMC counter passes (kernel-trace + pmc only; no sys/runtime traces) + repeated headline bench.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/pmc
mkdir -p $OUT
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
run() {  # run <name> <counters...>
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" -d $OUT/$name -o run --output-format csv -- \
    python bench.py --streams ${PMC_STREAMS:-8} --steps 20 --warmup 2 --cold-runs 0 > $OUT/$name.log 2>&1
  local rc=$?
  echo "pmc $name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
run A SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE
run B SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM
run C TCC_HIT_sum TCC_MISS_sum
python scripts/pmc_summary.py $OUT/A $OUT/B $OUT/C $OUT/pmc_summary.json
rm -rf $OUT/A $OUT/B $OUT/C
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 1000 --warmup 100 --cold-runs 0 > $OUT/bench_rep$i.log 2>&1 || exit $?
  grep -o '"value": [0-9.]*' $OUT/bench_rep$i.log
done
