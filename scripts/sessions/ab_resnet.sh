#!/bin/bash
# A/B of the ResNet-50 bs=1 bench between the repo (B) and a worktree build under ab/A (A),
# interleaved on ONE GPU box (box-to-box variance is larger than the effects measured).
set -u
OUT=${OUT:-gpurun_out/ab}
mkdir -p $OUT
run() {  # run <tag> <dir> <timeout> <cmd...>
  local tag=$1 dir=$2 to=$3; shift 3
  (cd $dir && timeout -k 10 $to "$@") > $OUT/$tag.log 2>&1
  local rc=$?
  echo "$tag rc=$rc $(grep -h '^{' $OUT/$tag.log | python3 -c 'import sys,json; [print(json.loads(l).get("value")) for l in sys.stdin]' 2>/dev/null)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP $tag rc=$rc"; exit $rc; fi
}
for X in A B; do
  D=$([ $X = A ] && echo ab/A || echo .)
  run tune_$X $D 600 python -m hipzap.engine.tune --model resnet50 --batch 1 --concurrent 1 8
done
for rep in 1 2; do
  for X in A B; do
    D=$([ $X = A ] && echo ab/A || echo .)
    run s1_${X}_$rep $D 300 python bench.py --streams 1 --steps 300 --warmup 30 --cold-runs 0
    run s8_${X}_$rep $D 300 python bench.py --streams 8 --steps 300 --warmup 30 --cold-runs 0
  done
done
