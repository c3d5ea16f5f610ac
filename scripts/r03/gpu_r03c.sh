#!/bin/bash
# Round-3 GPU pass C: bench contract (link probe on the shared card, cfg4,
# RCCL-init fallback), DDP / collective GPU tests (tune agreement), the
# reduce-role sweep over window memory kind / portion / workgroup size, then
# the IPC open A/B just below 2 GiB (last: stops at its first timeout).
set -o pipefail
mkdir -p gpurun_out/r03c
timeout -k 10 700 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_bench_contract_gpu.py tests/test_ddp_hook_gpu.py tests/test_collective_gpu.py > gpurun_out/r03c/pytest.log 2>&1 &&
timeout -k 10 300 python -u bench/ipc_reduce_role.py --n 8 --block-mb 32 --kinds fine,coarse,uncached --portion-kb 512,128 --threads 256,1024 --modes sys > gpurun_out/r03c/reduce_role_n8.jsonl 2>&1 &&
timeout -k 10 200 python -u bench/ipc_reduce_role.py --n 2,4 --block-mb 32 --kinds fine,coarse --portion-kb 512,128 --threads 1024 --modes sys > gpurun_out/r03c/reduce_role_n24.jsonl 2>&1 &&
AKKA_AB_CASES="coarse:2047,fine:2047" timeout -k 10 200 python -u scripts/ipc_open_ab.py > gpurun_out/r03c/ipc_open_ab.jsonl 2> gpurun_out/r03c/ipc_open_ab.err
