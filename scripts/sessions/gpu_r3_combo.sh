#!/bin/bash
set -u
bash scripts/gpu_r3_ab_conv.sh && bash scripts/gpu_r3_e2e.sh
