#!/bin/bash
# MX-fp8 GEMM per-config microbench on the ViT-B/16 bs64 shapes (+ a PMC pass over cfg 24 vs 43)
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/${TAG:-r3_mxb}
mkdir -p $O
timeout -k 10 300 python3 scripts/bench_mx.py > $O/bench_mx.jsonl 2> $O/bench_mx.err || { tail -5 $O/bench_mx.err; exit 1; }
python3 -c "
import json
for l in open('$O/bench_mx.jsonl'):
    d=json.loads(l); print(d['shape'], d['best_cfg'], d['best_us'], {k:v['us'] for k,v in d['cfgs'].items()})"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE GRBM_COUNT \
  -d $O/pmc1 -o run --output-format csv -- python3 scripts/bench_mx.py --cfgs 24,43,44 > $O/pmc1.log 2>&1 || { tail -5 $O/pmc1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_LDS \
  -d $O/pmc2 -o run --output-format csv -- python3 scripts/bench_mx.py --cfgs 24,43,44 > $O/pmc2.log 2>&1 || { tail -5 $O/pmc2.log; exit 1; }
for p in pmc1 pmc2; do python3 scripts/pmc_summary.py $O/$p $O/$p.json > /dev/null 2>&1; done
find $O -name "*.csv" -size +20M -delete
echo done
