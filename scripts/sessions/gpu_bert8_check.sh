set -o pipefail
o=gpurun_out/bert8; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_transformers_gpu.py -x -q --timeout 120 --timeout-method thread -k "bert" > $o/pytest.log 2>&1 || exit 1
timeout -k 10 400 python -m hipzap.engine.tune --model bert-base-fp8 --batch 16 --report $o/tune_report.json > $o/tune.log 2>&1 || exit 2
cp hipzap/tuning/bert-base-fp8_bs16.json $o/
timeout -k 10 300 python scripts/bench_models.py bert-base bert-base-fp8 > $o/models.jsonl 2>&1 || exit 3
