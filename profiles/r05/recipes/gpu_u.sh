#!/bin/bash
# Round-5 pass U: synchronous engine rounds record their input-ready marker
# only when a stream of the engine waits for it (none when the round runs on
# the caller's stream): host / per-round cost of small rounds (engine vs
# direct vs one-sided), then the GPU tests of the engine paths.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
O=gpurun_out/r05/u
mkdir -p $O
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 \
  --master-port 30301 profiles/r05/recipes/os_host_cost.py > $O/host.log 2>&1 || { echo "host rc=$?"; tail -20 $O/host.log; exit 1; }
grep lane $O/host.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_ipc_gpu.py tests/test_collective_gpu.py tests/test_stream_hazards_gpu.py tests/test_dp_ipc_gpu.py \
  tests/test_graph_step_gpu.py tests/test_cluster_ipc_gpu.py tests/test_ipc_p2p_gpu.py > $O/pytest.txt 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/pytest.txt | tail -8
exit $rc
