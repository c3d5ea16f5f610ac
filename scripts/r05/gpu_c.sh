#!/bin/bash
# Round-5 pass C: engine path with lane-written counts and caller-stream
# synchronous rounds (trace), then the GPU tests of the engine / ipc paths.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05/c
mkdir -p $O
bash scripts/r05/engine_path.sh engine_path_c > $O/engine_path.txt 2>&1 || { echo "engine path rc=$?"; tail -30 $O/engine_path.txt; exit 1; }
grep "run [0-9]\|^[0-9] \[" $O/engine_path.txt | head -40
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_ipc_gpu.py tests/test_collective_gpu.py tests/test_dp_ipc_gpu.py tests/test_ddp_hook_gpu.py \
  tests/test_graph_step_gpu.py tests/test_stream_hazards_gpu.py > $O/pytest.txt 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/pytest.txt | tail -20
exit $rc
