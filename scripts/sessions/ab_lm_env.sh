#!/bin/bash
# Same-box A/B of an environment variable on the AWD-LSTM decode (tests + per-kernel diag + bench).
#   bash scripts/ab_lm_env.sh OUTDIR VAR "v1 v2 ..."   (value "unset" = not set)
set -u
out=$1; var=$2; vals=$3
mkdir -p "$out"
for v in $vals; do
  if [ "$v" = unset ]; then pre=""; else pre="$var=$v"; fi
  env $pre timeout -k 10 200 python -u -m pytest tests/test_lm_gpu.py -x -q --timeout 120 --timeout-method thread > "$out/test_$v.log" 2>&1 || exit 1
  env $pre timeout -k 10 120 python -u scripts/diag_lm.py > "$out/diag_$v.json" 2>> "$out/err.log" || exit 1
  env $pre timeout -k 10 120 python -u scripts/bench_lm.py > "$out/bench_$v.json" 2>> "$out/err.log" || exit 1
done
