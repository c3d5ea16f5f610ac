#!/bin/bash
# tests/test_dp_ipc_gpu.py diagnosis: per-round out vs sum of inputs, by mode.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/dpdiag
export HSA_ENABLE_IPC_MODE_LEGACY=0
i=0
run() {  # run <n> <mode> <sync> <hwq>
  i=$((i+1)); d=$(mktemp -d)
  echo "== n=$1 mode=$2 sync=$3 hwq=$4"
  GPU_MAX_HW_QUEUES=$4 AKKA_DIAG_MODE=$2 AKKA_DIAG_SYNC=$3 timeout -k 10 150 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node=$1 --master-addr 127.0.0.1 --master-port $((29500 + i)) scripts/dp_ipc_diag.py $d 3 \
    > gpurun_out/dpdiag/run$i.log 2>&1
  local rc=$?
  grep -E "^step|^final|Error|error" gpurun_out/dpdiag/run$i.log | head -20
  return $rc
}
case "${DIAG:-hwq}" in
  modes) run 2 pull 0 4 && run 2 bcast 0 4 && run 2 pull 1 4 && run 3 pull 0 4 && run 2 fused 0 4 ;;
  hwq) run 2 pull 0 32 && run 3 pull 0 32 && run 2 pull 0 4 ;;
  pytest) timeout -k 10 400 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_dp_ipc_gpu.py -k dp_sgd 2>&1 | tail -15 ;;
esac
