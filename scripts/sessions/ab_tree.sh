#!/bin/bash
# Interleaved A/B of bench.py between the repo (B) and a worktree under ab/A (A), on ONE box,
# without retuning (same tuning tables): isolates a kernel change. TREES="ab/A ab/C ." compares
# more variants (each a pre-built tree).
#   REPS=2 STREAMS="1 8" bash scripts/ab_tree.sh
set -u
OUT=${OUT:-gpurun_out/ab_tree}
mkdir -p $OUT
for rep in $(seq 1 ${REPS:-2}); do
  for D in ${TREES:-ab/A .}; do
    X=$(basename $(cd $D && pwd))
    for s in ${STREAMS:-1 8}; do
      log=$OUT/${X}_s${s}_$rep.log
      (cd $D && timeout -k 10 300 python bench.py --streams $s --steps ${STEPS:-300} --warmup 30 --cold-runs 0) > $log 2>&1
      rc=$?
      echo "$X s$s rep$rep rc=$rc $(grep -h '^{' $log | python3 -c 'import sys,json; [print(json.loads(l).get("value"), json.loads(l).get("latency_ms_p50_single")) for l in sys.stdin]' 2>/dev/null)"
      if [ $rc -ne 0 ]; then echo "STOP $X rc=$rc"; tail -5 $log; exit $rc; fi
    done
  done
done
