#!/bin/bash
# Same-box A/B of an environment variable on scripts/bench_models.py (interleaved, 2 runs each).
#   bash scripts/ab_models_env.sh OUTDIR VAR "v1 v2 ..."   (value "unset" = not set)
set -u
out=$1; var=$2; vals=$3
mkdir -p "$out"
for v in $vals $vals; do
  if [ "$v" = unset ]; then pre=""; else pre="$var=$v"; fi
  env $pre timeout -k 10 300 python -u scripts/bench_models.py >> "$out/b_$v.jsonl" 2>> "$out/err.log" || exit 1
done
