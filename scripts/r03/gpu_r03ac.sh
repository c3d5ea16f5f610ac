#!/bin/bash
# Round-3 GPU pass AC: bench contract tests (extras on the headline's
# transport, config-3-sized ipc windows, preflight fallback to the ipc lanes),
# DDP hook tests, and the MLP example with the graphed step.
set -o pipefail
mkdir -p gpurun_out/r03ac
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_bench_contract_gpu.py \
  tests/test_ddp_hook_gpu.py > gpurun_out/r03ac/pytest.log 2>&1 &&
timeout -k 10 200 python -u examples/mlp_sgd.py --compute-dtype bfloat16 --graph --steps 200 --warmup 20 \
  > gpurun_out/r03ac/mlp_sgd_graph.json 2> gpurun_out/r03ac/mlp_sgd_graph.err
