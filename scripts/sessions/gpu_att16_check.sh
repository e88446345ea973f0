set -o pipefail
o=gpurun_out/att16; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_transformers_gpu.py tests/test_fp8_gpu.py -x -q --timeout 120 --timeout-method thread > $o/pytest.log 2>&1 || exit 1
for v in 0 1 0 1; do
  HIPZAP_ATT_NW16=$v timeout -k 10 200 python bench.py --mode scatter --model vit-b16-fp8 --global-batch 64 --steps 50 --warmup 5 --cold-trials 0 > $o/scatter_nw16_$v.$RANDOM.log 2>&1 || exit 2
done
for v in 0 1; do
  HIPZAP_ATT_NW16=$v timeout -k 10 200 python scripts/bench_models.py vit-b16-fp8 vit-b16 > $o/models_nw16_$v.jsonl 2>&1 || exit 3
done
