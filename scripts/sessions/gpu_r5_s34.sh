#!/bin/bash
# r5 s34: AWD-LSTM one-request program, tiles per layer workgroup (HIPZAP_LMB_SOLO unset = round 4,
# t2 / t3 = two / three tiles for every layer): bitwise tests, interleaved A/B
# (lone request, 32 / 64 clients)
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5_s34; mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 180 --timeout-method thread -m gpu tests/test_lmbatch_gpu.py tests/test_lmlite_gpu.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"
grep -E 'FAILED|ERROR|passed|failed' $O/pytest.log | tail -25
[ $rc -le 1 ] || exit 1
for sh in t2 t3; do
  HIPZAP_LMB_SOLO=$sh timeout -k 10 300 python -u -m pytest -q --timeout 180 --timeout-method thread -m gpu tests/test_lmbatch_gpu.py -k "one_request" > $O/pytest_$sh.log 2>&1
  rc=$?; echo "pytest $sh rc=$rc $(tail -1 $O/pytest_$sh.log)"
  [ $rc -le 1 ] || exit 1
done
for rep in 1 2; do
  for sh in r4 t2 t3; do
    HIPZAP_LMB_SOLO=$([ $sh = r4 ] && echo "" || echo $sh) timeout -k 10 300 python3 scripts/bench_lm_batch.py --clients 1 32 64 --requests 12 > $O/lm_${sh}_$rep.json 2> $O/lm_${sh}_$rep.err || { tail -20 $O/lm_${sh}_$rep.err; exit 1; }
    python3 -c "
import json; j=json.loads(open('$O/lm_${sh}_$rep.json').read().strip().splitlines()[-1])
print('solo=$sh rep $rep single', j['single_request_ms'], j['single_us_per_step'], [(l['clients'], l['req_per_s'], l['us_per_step'], l['p50_ms']) for l in j['load']])"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/p1 -o run -- python3 scripts/bench_lm_batch.py --clients 1 --requests 4 > $O/prof_c1.log 2>&1 || { tail -20 $O/prof_c1.log; exit 1; }
db=$(find $O/p1 -name '*results.db' | head -1)
python3 scripts/rocpd_stats.py "$db" 20 > $O/kernel_stats_c1.txt
rm -rf $O/p1
cut -c1-150 $O/kernel_stats_c1.txt | head -12
