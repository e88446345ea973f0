set -o pipefail
o=gpurun_out/bs1tune; mkdir -p $o
cp hipzap/tuning/resnet50_bs1.json $o/old_bs1.json; cp hipzap/tuning/resnet50_bs1_c24.json $o/old_bs1_c24.json
timeout -k 10 200 python bench.py --cold-trials 0 --cold-runs 0 --dyn-batch 0 > $o/bench_old_a.log 2>&1 || exit 1
timeout -k 10 500 python -m hipzap.engine.tune --batch 1 --concurrent 1 24 --report $o/tune_report.json > $o/tune.log 2>&1 || exit 2
cp hipzap/tuning/resnet50_bs1.json $o/new_bs1.json; cp hipzap/tuning/resnet50_bs1_c24.json $o/new_bs1_c24.json
timeout -k 10 200 python bench.py --cold-trials 0 --cold-runs 0 --dyn-batch 0 > $o/bench_new_a.log 2>&1 || exit 3
cp $o/old_bs1.json hipzap/tuning/resnet50_bs1.json; cp $o/old_bs1_c24.json hipzap/tuning/resnet50_bs1_c24.json
timeout -k 10 200 python bench.py --cold-trials 0 --cold-runs 0 --dyn-batch 0 > $o/bench_old_b.log 2>&1 || exit 4
cp $o/new_bs1.json hipzap/tuning/resnet50_bs1.json; cp $o/new_bs1_c24.json hipzap/tuning/resnet50_bs1_c24.json
timeout -k 10 200 python bench.py --cold-trials 0 --cold-runs 0 --dyn-batch 0 > $o/bench_new_b.log 2>&1 || exit 5
