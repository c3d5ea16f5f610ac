#!/bin/bash
# Round-5 pass B: engine path after the fix (trace), then the GPU tests of the
# changed parts (one-sided hand-off modes, direct ipc lanes, graphs, engine
# path, bench contract).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05/b
mkdir -p $O
bash scripts/r05/engine_path.sh engine_path_after > $O/engine_path.txt 2>&1 || { echo "engine path rc=$?"; tail -30 $O/engine_path.txt; exit 1; }
grep "run [0-9]" $O/engine_path.txt | head -20
timeout -k 10 1000 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_ipc_gpu.py tests/test_onesided_gpu.py tests/test_graph_step_gpu.py tests/test_collective_gpu.py \
  tests/test_bench_contract_gpu.py tests/test_cluster_onesided_gpu.py > $O/pytest.txt 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest.txt | tail -80
exit $rc
