#!/bin/bash
# Round-3 GPU pass B: ipc lane tests (late rank poisons the round, templated
# reduce), mailbox p2p tests (residency-capped grid), the reduce-role
# microbenchmark and its raw TCC counters, then the IPC open A/B (last: it
# stops at its first timeout).
set -o pipefail
mkdir -p gpurun_out/r03b
timeout -k 10 700 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_ipc_gpu.py tests/test_ipc_p2p_gpu.py > gpurun_out/r03b/pytest_ipc.log 2>&1 &&
timeout -k 10 300 python -u bench/ipc_reduce_role.py --n 2,4,8 --block-mb 4,32 --threads 256,1024 > gpurun_out/r03b/reduce_role.jsonl 2>&1 &&
timeout -k 10 400 bash scripts/pmc_ipc_reduce.sh > gpurun_out/r03b/pmc.log 2>&1 &&
AKKA_AB_CASES="coarse:2048,coarse:2560,coarse:4096,fine:2048,fine:2560" timeout -k 10 400 python -u scripts/ipc_open_ab.py > gpurun_out/r03b/ipc_open_ab.jsonl 2> gpurun_out/r03b/ipc_open_ab.err
