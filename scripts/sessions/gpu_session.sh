#!/bin/bash
# One gpurun session: GPU tests, smoke, bench variants, rocprof kernel stats.
# Continues past ordinary test failures (rc 1) but stops at any crash/timeout/fault.
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 5 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-all}
python -c "import torch; print(torch.cuda.get_device_name(0))"
[[ $STEPS == *tests* || $STEPS == all ]] && step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
[[ $STEPS == *smoke* || $STEPS == all ]] && step smoke 300 python __graft_entry__.py smoke
[[ $STEPS == *tune* || $STEPS == all ]] && {
  step tune 900 python -m hipzap.engine.tune --model ${TUNE_MODEL:-resnet50} --batch ${TUNE_BATCH:-1} --concurrent ${TUNE_CONC:-1 8} --report $OUT/tune_report.json
  mkdir -p $OUT/tuning && cp hipzap/tuning/*.json $OUT/tuning/
}
[[ $STEPS == *txtune* ]] && {
  step txtune_bert 600 python -m hipzap.engine.tune --model bert-base --batch 16 --report $OUT/tune_bert.json
  step txtune_vit 600 python -m hipzap.engine.tune --model vit-b16 --batch 8 --report $OUT/tune_vit.json
  step txtune_vit8 600 python -m hipzap.engine.tune --model vit-b16-fp8 --batch 8 --report $OUT/tune_vit8.json
  mkdir -p $OUT/tuning && cp hipzap/tuning/*.json $OUT/tuning/
}
[[ $STEPS == *models* ]] && step bench_models 900 python scripts/bench_models.py
[[ $STEPS == *lm* ]] && step bench_lm 600 python scripts/bench_lm.py
[[ $STEPS == *bench* || $STEPS == all ]] && {
  for s in ${BENCH_STREAMS:-1 4 8}; do
    step bench_s$s 300 python bench.py --streams $s --steps 300 --warmup 30 --cold-runs 2 ${BENCH_EXTRA:-}
    grep '^{' $OUT/bench_s$s.log > $OUT/bench_s$s.json || true
  done
}
[[ $STEPS == *" prof"* || $STEPS == prof* || $STEPS == all ]] && {
  step rocprof 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --streams 1 --steps 50 --warmup 5 --cold-runs 0
  python scripts/trace_summary.py $OUT/prof $OUT/prof_summary && rm -rf $OUT/prof
}
[[ $STEPS == *txprof* ]] && {
  for mb in "bert-base 16" "vit-b16 8" "vit-b16-fp8 8"; do
    set -- $mb
    step prof_$1 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$1 -o run --output-format csv -- python3 scripts/prof_model.py --model $1 --batch $2 --iters 20
    python scripts/trace_summary.py $OUT/prof_$1 $OUT/prof_summary_$1; rm -rf $OUT/prof_$1
  done
}
[[ $STEPS == *lmprof* ]] && {
  export HIPZAP_LM_WORDS=50 HIPZAP_LM_CONTEXTS=1
  step prof_lm 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_lm -o run --output-format csv -- python3 scripts/bench_lm.py
  python scripts/trace_summary.py $OUT/prof_lm $OUT/prof_summary_lm lstm_cell_kernel; rm -rf $OUT/prof_lm
}
echo "=== done"
