#!/bin/bash
# Round-3 GPU pass AE: graphed bf16 step with a bf16 static input buffer.
set -o pipefail
mkdir -p gpurun_out/r03ae
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_step_gpu.py \
  > gpurun_out/r03ae/pytest.log 2>&1 &&
for i in 1 2; do
  timeout -k 10 120 python -u bench/cfg5_step.py --dtype bf16 --graph --steps 500 --warmup 50 >> gpurun_out/r03ae/cfg5.jsonl 2>/dev/null || exit 1
done
