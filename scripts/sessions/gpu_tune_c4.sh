set -o pipefail
o=gpurun_out/c4; mkdir -p $o
timeout -k 10 300 python scripts/bench_models.py bert-base bert-base-fp8 vit-b16-fp8 > $o/models_old.jsonl 2>&1 || exit 1
for m in bert-base:16 bert-base-fp8:16 vit-b16-fp8:8; do
  timeout -k 10 400 python -m hipzap.engine.tune --model ${m%%:*} --batch ${m##*:} --concurrent 4 --report $o/tune_${m%%:*}.json > $o/tune_${m%%:*}.log 2>&1 || exit 2
  cp hipzap/tuning/${m%%:*}_bs${m##*:}_c4.json $o/
done
timeout -k 10 300 python scripts/bench_models.py bert-base bert-base-fp8 vit-b16-fp8 > $o/models_new.jsonl 2>&1 || exit 3
