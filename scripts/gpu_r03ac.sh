#!/bin/bash
# Round-3 GPU pass AC: bench contract tests after the extras share the
# headline's transport and its config-3-sized ipc windows.
set -o pipefail
mkdir -p gpurun_out/r03ac
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_bench_contract_gpu.py \
  tests/test_ddp_hook_gpu.py > gpurun_out/r03ac/pytest.log 2>&1
