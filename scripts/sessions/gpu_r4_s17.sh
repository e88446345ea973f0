#!/bin/bash
# r4: BERT-base bs16 LayerNorm fold (experiments build) vs the lean build, interleaved, + kernel stats
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4_s17; mkdir -p $O
EXP=$PWD/hipzap/_lib/libhipzap_exp.so
for rep in 1 2; do
  for v in expfold1 expfold0 lean0; do
    case $v in
      expfold1) env_="HIPZAP_LIB=$EXP HIPZAP_LN_FOLD=1";;
      expfold0) env_="HIPZAP_LIB=$EXP HIPZAP_LN_FOLD=0";;
      lean0) env_="HIPZAP_LN_FOLD=0";;
    esac
    env $env_ timeout -k 10 300 python scripts/bench_models.py bert-base > $O/${v}_$rep.log 2>&1 || { tail -20 $O/${v}_$rep.log; exit 1; }
    echo "$v rep$rep $(grep -h '^{' $O/${v}_$rep.log | tr '\n' ' ')"
  done
done
HIPZAP_LIB=$EXP HIPZAP_LN_FOLD=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof1 -o run -- python3 scripts/bench_models.py bert-base > $O/prof1.log 2>&1 || { tail -20 $O/prof1.log; exit 1; }
HIPZAP_LN_FOLD=0 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof0 -o run -- python3 scripts/bench_models.py bert-base > $O/prof0.log 2>&1 || { tail -20 $O/prof0.log; exit 1; }
ls -R $O | head -30
