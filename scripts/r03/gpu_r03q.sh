#!/bin/bash
# Round-3 GPU pass Q: column sum after the one-latency combine and 8 rows in
# flight; config-5 step A/B (bf16 weight shadow on / off) on one box.
set -o pipefail
mkdir -p gpurun_out/r03q
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fused_step_gpu.py \
  > gpurun_out/r03q/pytest.log 2>&1 &&
timeout -k 10 200 python -u bench/colsum_bw.py > gpurun_out/r03q/colsum.jsonl 2> gpurun_out/r03q/colsum.err &&
timeout -k 10 200 python -u bench/cfg5_step.py --dtype bf16 --no-shadow > gpurun_out/r03q/cfg5.jsonl 2>&1 &&
timeout -k 10 200 python -u bench/cfg5_step.py --dtype bf16 >> gpurun_out/r03q/cfg5.jsonl 2>&1 &&
timeout -k 10 200 python -u bench/cfg5_step.py --dtype bf16 --no-shadow >> gpurun_out/r03q/cfg5.jsonl 2>&1 &&
timeout -k 10 200 python -u bench/cfg5_step.py --dtype bf16 >> gpurun_out/r03q/cfg5.jsonl 2>&1
