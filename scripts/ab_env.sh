#!/bin/bash
# Same-box A/B of an environment variable on the serving bench (interleaved runs).
#   bash scripts/ab_env.sh OUTDIR VAR "v1 v2 ..." [bench args...]   (value "unset" = not set)
set -u
out=$1; var=$2; vals=$3; shift 3
mkdir -p "$out"
for v in $vals $vals; do
  if [ "$v" = unset ]; then
    timeout -k 10 200 python bench.py "$@" >> "$out/$v.jsonl" 2>> "$out/err.log" || exit 1
  else
    env "$var=$v" timeout -k 10 200 python bench.py "$@" >> "$out/$v.jsonl" 2>> "$out/err.log" || exit 1
  fi
done
