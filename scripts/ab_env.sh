#!/bin/bash
# Interleaved A/B of bench.py under different environment settings on ONE box:
#   VARIANTS="base:  zc:HIPZAP_ZERO_COPY=all" STREAMS="1 8" REPS=2 bash scripts/ab_env.sh
# (box-to-box variance is larger than most effects; only same-box interleaved runs compare)
set -u
OUT=${OUT:-gpurun_out/ab_env}
mkdir -p $OUT
for rep in $(seq 1 ${REPS:-2}); do
  for v in ${VARIANTS}; do
    tag=${v%%:*}; envs=${v#*:}
    for s in ${STREAMS:-1 8}; do
      log=$OUT/${tag}_s${s}_$rep.log
      env $(echo $envs | tr ',' ' ') timeout -k 10 300 python bench.py --streams $s --steps ${STEPS:-300} --warmup 30 --cold-runs 0 ${EXTRA:-} > $log 2>&1
      rc=$?
      echo "$tag s$s rep$rep rc=$rc $(grep -h '^{' $log | python3 -c 'import sys,json; [print(json.loads(l).get("value"), json.loads(l).get("latency_ms_p50_single")) for l in sys.stdin]' 2>/dev/null)"
      if [ $rc -ne 0 ]; then echo "STOP $tag rc=$rc"; tail -5 $log; exit $rc; fi
    done
  done
done
