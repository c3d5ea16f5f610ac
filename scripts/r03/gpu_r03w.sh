#!/bin/bash
# Round-3 GPU pass W: one-source big-stream pass at unroll 4 / 2 blocks per CU:
# kernel tests, the sweep point, bench.py N=1 (headline + cfg3).
set -o pipefail
mkdir -p gpurun_out/r03w
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_collective_gpu.py > gpurun_out/r03w/pytest.log 2>&1 &&
timeout -k 10 120 python -u bench/n1_bigcopy.py 1073741824 bf16 > gpurun_out/r03w/bigcopy.jsonl 2>/dev/null &&
timeout -k 10 300 python bench.py > gpurun_out/r03w/bench_n1.json 2> gpurun_out/r03w/bench_n1.err
