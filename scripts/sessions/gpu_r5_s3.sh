#!/bin/bash
# r5 s3: where the seam program's time goes -- per-position kernel durations, 1 and 16 streams
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5_s3; mkdir -p $O
B="--cold-trials 0 --cold-runs 0 --http-clients 0 --dp-figures 0 --dyn-batch 0 --bert-cold 0 --lm-cold 0"
for v in seam seam128; do
  case $v in
    seam) CS=128,64;;
    seam128) CS=128,128;;
  esac
  for s in 1 16; do
    HIPZAP_FUSE=convpool,bneck,bneck2,seam HIPZAP_SEAM_CS=$CS timeout -k 10 300 rocprofv3 --kernel-trace -d $O/p -o run -- python3 bench.py --streams $s --steps 60 --warmup 5 $B > $O/prof_${v}_$s.log 2>&1 || { tail -20 $O/prof_${v}_$s.log; exit 1; }
    python3 scripts/rocpd_stats.py $O/p/run_results.db --cutime preprocess pool_fc > $O/cutime_${v}_$s.txt
    rm -rf $O/p
  done
done
tail -33 $O/cutime_seam_1.txt
