#!/bin/bash
# Plan weight-upload sub-phases over fresh processes (HIPZAP_PLAN_PROBE=2 prints them to stderr).
set -e
mkdir -p gpurun_out/up
timeout -k 10 120 python -c "
import sys; sys.path.insert(0, '.')
from bench import prepare_artifacts
print(prepare_artifacts('resnet50', '/tmp/hipzap_bench')[1])" > gpurun_out/up/plan_path.txt 2> gpurun_out/up/prep.err
for i in 1 2 3 4 5; do
  HIPZAP_PLAN_PROBE=2 timeout -k 10 60 python -c "
import sys, json; sys.path.insert(0, '.')
from hipzap.lite import PlanEngine
e = PlanEngine(open('gpurun_out/up/plan_path.txt').read().strip(), device=0, contexts=1)
print(json.dumps({k: round(v, 2) for k, v in e.timings.items()}))" >> gpurun_out/up/phases.jsonl 2>> gpurun_out/up/upload.log
done
