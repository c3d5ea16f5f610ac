#!/bin/bash
# Round-3 GPU pass R: the whole GPU suite on this tree (what the driver runs
# at round end), then config-5 A/B with longer runs, alternating.
set -o pipefail
mkdir -p gpurun_out/r03r
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/r03r/pytest_gpu.log 2>&1 &&
for i in 1 2; do
  timeout -k 10 120 python -u bench/cfg5_step.py --dtype bf16 --no-shadow --steps 500 --warmup 50 >> gpurun_out/r03r/cfg5.jsonl 2>/dev/null &&
  timeout -k 10 120 python -u bench/cfg5_step.py --dtype bf16 --steps 500 --warmup 50 >> gpurun_out/r03r/cfg5.jsonl 2>/dev/null || exit 1
done
