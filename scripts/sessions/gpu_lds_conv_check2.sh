set -o pipefail
O=gpurun_out/lds2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_conv_lds_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --mode scatter --global-batch 32 --steps 100 --warmup 10 --cold-trials 0 --tuned scripts/empty_tuning.json > $O/scatter_heur.log 2>&1 || exit 3
for b in 4 8 16; do cp hipzap/tuning/resnet50_bs$b.json $O/resnet50_bs${b}_old.json 2>/dev/null; done
timeout -k 10 500 python -m hipzap.engine.tune --batch 4 8 16 --report $O/tune_report.json > $O/tune.log 2>&1 || exit 4
for b in 4 8 16; do cp hipzap/tuning/resnet50_bs$b.json $O/resnet50_bs${b}_new.json; done
for b in 4 8 16; do
  timeout -k 10 200 python bench.py --batch $b --streams 4 --steps 200 --warmup 20 --cold-trials 0 > $O/replica_bs${b}_s4.log 2>&1 || exit 5
done
timeout -k 10 200 python bench.py --batch 8 --streams 8 --steps 200 --warmup 20 --cold-trials 0 > $O/replica_bs8_s8.log 2>&1 || exit 6
