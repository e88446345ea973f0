#!/bin/bash
# r4 diagnostics for the next round: what the LM decoder's state staging and its lo-half
# MFMAs / LDS reads cost at 32 rows (experiments build, timing-only variants: garbage tokens)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_s25; mkdir -p $O
export HIPZAP_LIB=$PWD/hipzap/_lib/libhipzap_exp.so
for rep in 1 2; do
for d in 0 1 2; do
  HIPZAP_LM_SOLO=0 HIPZAP_LMB_DEC_DIAG=$d timeout -k 10 200 python scripts/bench_lm_batch.py --clients 1 32 --requests 10 > $O/lm_diag${d}_$rep.json 2> $O/lm_err.log || { tail -20 $O/lm_err.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/lm_diag${d}_$rep.json').read().strip().splitlines()[-1]); print('diag=$d rep$rep', [(l['clients'], l['us_per_step']) for l in d['load']])"
done
done
