#!/bin/bash
# Round-3 GPU pass A: one-sided lane tests (kept records), bench contract tests
# (ipc / ipc_p2p flows, cfg4 on the one-sided lane, RCCL-init fallback), an
# N=1 bench line, then the risky steps last: the straggler-kill test and the
# IPC open A/B (stops at its first timeout).
set -o pipefail
mkdir -p gpurun_out/r03a
export AKKA_TEST_KEEP=gpurun_out/r03a/onesided
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_onesided_gpu.py -k "not killed" tests/test_bench_contract_gpu.py > gpurun_out/r03a/pytest.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --extras off > gpurun_out/r03a/bench_n1.json 2> gpurun_out/r03a/bench_n1.err &&
timeout -k 10 240 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_onesided_gpu.py -k killed > gpurun_out/r03a/pytest_kill.log 2>&1 &&
timeout -k 10 400 python -u scripts/ipc_open_ab.py > gpurun_out/r03a/ipc_open_ab.jsonl 2> gpurun_out/r03a/ipc_open_ab.err
