#!/bin/bash
# Round-5 pass N: per-role timeline of the one-sided round (AKKA_OS_TIMELINE),
# 4 ranks on the card, 64 / 256 MiB, gather copy vs window output; then the
# DDP GPU tests (shared masked stream assertion).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
O=gpurun_out/r05/n
mkdir -p $O/copy $O/wo
timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node=4 --master-addr 127.0.0.1 \
  --master-port 29931 bench/onesided_timeline.py --out-dir $O/copy > $O/copy.log 2>&1 || { echo "copy rc=$?"; tail -20 $O/copy.log; exit 1; }
timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node=4 --master-addr 127.0.0.1 \
  --master-port 29932 bench/onesided_timeline.py --window-output --out-dir $O/wo > $O/wo.log 2>&1 || { echo "wo rc=$?"; tail -20 $O/wo.log; exit 1; }
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_dp_ipc_gpu.py -k onesided > $O/pytest.txt 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/pytest.txt | tail -8
exit $rc
