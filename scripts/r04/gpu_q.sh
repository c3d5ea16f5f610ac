#!/bin/bash
# Round-4 pass Q: DDP with the one-sided hook, sync vs async bucket rounds
# (2 processes on the card, cu_keep 6), plus the async exact-round GPU test.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r04q
mkdir -p $O
AKKA_SHARE_GPU=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=2 \
  --master-addr 127.0.0.1 --master-port 29771 bench/ddp_overlap.py > $O/ddp.log 2>&1 \
  || { echo "ddp rc=$?"; grep -v Warning $O/ddp.log | tail -30; exit 1; }
grep '^{' $O/ddp.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_onesided_gpu.py -k async \
  tests/test_dp_ipc_gpu.py tests/test_ddp_hook_gpu.py > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
