#!/bin/bash
# Round-3 GPU pass AK: the fused average + SGD + shadow pass's grid, alternating.
set -o pipefail
mkdir -p gpurun_out/r03ak
for i in 1 2; do
  for g in 2048 4096 8192 16384 32768; do
    env AKKA_CM_MAXGRID=$g timeout -k 10 120 python -u bench/sgd_pass_bw.py >> gpurun_out/r03ak/sweep.jsonl 2>/dev/null || exit 1
  done
done
