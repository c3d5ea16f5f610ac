#!/bin/bash
# Round-3 GPU pass AJ: N=1 headline with one-source passes at 64 blocks/CU:
# kernel + collective tests, bench.py N=1 twice, the pass alone.
set -o pipefail
mkdir -p gpurun_out/r03aj
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_collective_gpu.py tests/test_fused_step_gpu.py > gpurun_out/r03aj/pytest.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/r03aj/bench_n1_a.json 2> gpurun_out/r03aj/bench_n1_a.err &&
timeout -k 10 300 python bench.py --extras off --steps 50 > gpurun_out/r03aj/bench_n1_b.json 2> gpurun_out/r03aj/bench_n1_b.err &&
timeout -k 10 120 python -u bench/n1_bigcopy.py 268435456 fp32 > gpurun_out/r03aj/pass.jsonl 2>/dev/null
