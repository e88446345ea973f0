#!/bin/bash
# Round 3 transformer baseline on one MI355X: GEMM microbench vs hipBLASLt; same-box interleaved
# A/B of BERT / ViT model benches (base = hipzap/_lib/base/libhipzap_base.so, new = in-tree);
# ViT-fp8 config-5 scatter bench; rocprof kernel stats of BERT bs16 and ViT-fp8 bs64 (new).
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/${TAG:-r3_tx_base}
mkdir -p $O
timeout -k 10 300 python3 scripts/bench_gemm.py > $O/gemm.jsonl 2> $O/gemm.err || { tail -5 $O/gemm.err; exit 1; }
for rep in 1 2; do
  for v in base new; do
    if [ $v = base ]; then export HIPZAP_LIB=hipzap/_lib/base/libhipzap_base.so; else unset HIPZAP_LIB; fi
    timeout -k 10 400 python3 scripts/bench_models.py ${MODELS:-bert-base vit-b16-fp8} > $O/models_${v}_$rep.jsonl 2> $O/models_${v}_$rep.err \
      || { tail -5 $O/models_${v}_$rep.err; exit 1; }
    echo "$v $rep: $(cut -c1-100 $O/models_${v}_$rep.jsonl | tr '\n' ' ')"
  done
done
unset HIPZAP_LIB
timeout -k 10 300 python3 bench.py --mode scatter --model vit-b16-fp8 --global-batch 64 --steps 50 --warmup 5 \
  --cold-trials 0 --cold-runs 0 > $O/vit64.log 2>&1 || { tail -5 $O/vit64.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_bert -o run --output-format csv -- \
  python3 scripts/prof_model.py --model bert-base --batch 16 --iters 20 > $O/prof_bert.log 2>&1 || { tail -5 $O/prof_bert.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_vit64 -o run --output-format csv -- \
  python3 scripts/prof_model.py --model vit-b16-fp8 --batch 64 --iters 10 > $O/prof_vit64.log 2>&1 || { tail -5 $O/prof_vit64.log; exit 1; }
find $O -name "*kernel_trace.csv" -delete
tail -2 $O/vit64.log
echo done
