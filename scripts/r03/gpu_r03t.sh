#!/bin/bash
# Round-3 GPU pass T: graphed config-5 step without captured fills / copies;
# bench contract; N=1 bench line.
set -o pipefail
mkdir -p gpurun_out/r03t
R=$(pwd)
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_fused_step_gpu.py \
  tests/test_bench_contract_gpu.py > gpurun_out/r03t/pytest.log 2>&1 &&
timeout -k 10 120 python -u bench/cfg5_step.py --dtype bf16 --graph --steps 500 --warmup 50 > gpurun_out/r03t/cfg5.jsonl 2>/dev/null &&
timeout -k 10 120 python -u bench/cfg5_step.py --dtype bf16 --steps 500 --warmup 50 >> gpurun_out/r03t/cfg5.jsonl 2>/dev/null &&
timeout -k 10 300 python bench.py > gpurun_out/r03t/bench_n1.json 2> gpurun_out/r03t/bench_n1.err &&
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d $R/gpurun_out/r03t/cfg5_trace -o run -- python3 $R/bench/cfg5_step.py --dtype bf16 --graph --steps 30 \
  > $R/gpurun_out/r03t/cfg5_trace.log 2>&1)
