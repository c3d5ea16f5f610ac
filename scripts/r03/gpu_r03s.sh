#!/bin/bash
# Round-3 GPU pass S: fused cross entropy + graphed forward/backward for the
# config-5 step: tests, then eager-baseline / eager-fused / graphed A/B
# (500 steps, interleaved twice), kernel stats of the graphed step.
set -o pipefail
mkdir -p gpurun_out/r03s
R=$(pwd)
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fused_step_gpu.py \
  tests/test_collective_gpu.py > gpurun_out/r03s/pytest.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 120 python -u bench/cfg5_step.py --dtype bf16 --no-shadow --no-fused-loss --steps 500 --warmup 50 >> gpurun_out/r03s/cfg5.jsonl 2>/dev/null &&
  timeout -k 10 120 python -u bench/cfg5_step.py --dtype bf16 --steps 500 --warmup 50 >> gpurun_out/r03s/cfg5.jsonl 2>/dev/null &&
  timeout -k 10 120 python -u bench/cfg5_step.py --dtype bf16 --graph --steps 500 --warmup 50 >> gpurun_out/r03s/cfg5.jsonl 2>/dev/null &&
  timeout -k 10 120 python -u bench/cfg5_step.py --dtype fp32 --graph --steps 500 --warmup 50 >> gpurun_out/r03s/cfg5.jsonl 2>/dev/null || exit 1
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d $R/gpurun_out/r03s/cfg5_trace -o run -- python3 $R/bench/cfg5_step.py --dtype bf16 --graph --steps 30 \
  > $R/gpurun_out/r03s/cfg5_trace.log 2>&1)
