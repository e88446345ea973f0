#!/bin/bash
# r6 session 1: determinism + seam tests, exclusive-CU A/B (HIPZAP_EXCL_LDS), probes.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r6_s1
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_determinism_gpu.py tests/test_seam_gpu.py > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 $OUT/tests.log
[ $rc -le 1 ] || exit $rc
B="python3 bench.py --cold-trials 0 --dyn-batch 0 --http-clients 0 --dp-figures 0 --config-figures 0 --cold-runs 0 --steps 20 --warmup 5"
for rep in 1 2; do
  for v in 0 83000; do
    HIPZAP_EXCL_LDS=$v timeout -k 10 180 $B > $OUT/ab_excl${v}_rep$rep.log 2>&1
    rc=$?; echo "ab excl=$v rep=$rep rc=$rc"
    [ $rc -eq 0 ] || { tail -5 $OUT/ab_excl${v}_rep$rep.log; exit $rc; }
    grep '^{' $OUT/ab_excl${v}_rep$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(' value', d['value'], 'sustained', d['served_sustained']['inf_s'], 'p50_single', d['latency_ms_p50_single'])"
  done
done
bash scripts/sessions/r6_probe.sh
