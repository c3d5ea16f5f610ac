#!/bin/bash
# Round-3 GPU pass E: reduce-role sweep (portion x workgroup size x grid cap,
# fenced vs lite hand-offs; kernels per rank count, nontemporal output
# stores), then the ipc lane tests (incl. the config-3 window) and the
# onesided tests after the per-N reduce kernels.
set -o pipefail
mkdir -p gpurun_out/r03e
timeout -k 10 300 python -u bench/ipc_reduce_role.py --n 8 --block-mb 32 --kinds fine --portion-kb 256,512,1024 \
  --threads 256,1024 --max-wgs 1024,2048,4096 --modes sys,lite > gpurun_out/r03e/reduce_role_sweep_n8.jsonl 2>&1 &&
timeout -k 10 200 python -u bench/ipc_reduce_role.py --n 2,4 --block-mb 32 --kinds fine --portion-kb 512,1024 \
  --threads 256,1024 --max-wgs 1024,4096 --modes sys,lite > gpurun_out/r03e/reduce_role_sweep_n24.jsonl 2>&1 &&
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_ipc_gpu.py tests/test_onesided_gpu.py > gpurun_out/r03e/pytest.log 2>&1
