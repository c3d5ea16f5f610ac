#!/bin/bash
# Round-3 GPU pass P: bias-gradient column-sum variants (write-through vs
# fenced partial-row hand-off, row splits) alone and behind the dW GEMM;
# config-5 step with the chosen variant; colsum GPU tests.
set -o pipefail
mkdir -p gpurun_out/r03p
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fused_step_gpu.py \
  > gpurun_out/r03p/pytest.log 2>&1 &&
timeout -k 10 200 python -u bench/colsum_bw.py > gpurun_out/r03p/colsum.jsonl 2> gpurun_out/r03p/colsum.err &&
timeout -k 10 200 python -u bench/cfg5_step.py --dtype bf16 > gpurun_out/r03p/cfg5.jsonl 2>&1
