#!/bin/bash
# Round-3 GPU pass D: ipc lane tests after the shared-window refactor (incl.
# the lite hand-offs), DDP hook on one transport / one window set, onesided,
# then the reduce-role sweep sys vs lite hand-offs.
set -o pipefail
mkdir -p gpurun_out/r03d
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_ipc_gpu.py tests/test_ipc_p2p_gpu.py tests/test_dp_ipc_gpu.py > gpurun_out/r03d/pytest_ipc.log 2>&1 &&
timeout -k 10 300 python -u bench/ipc_reduce_role.py --n 2,8 --block-mb 32 --kinds fine --portion-kb 512 --threads 1024 --modes sys,lite > gpurun_out/r03d/reduce_role_lite.jsonl 2>&1 &&
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_onesided_gpu.py tests/test_cluster_ipc_gpu.py > gpurun_out/r03d/pytest_os.log 2>&1
