#!/bin/bash
# enable_ipc cost vs window size and memory kind (processes sharing the card)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ipc_open
i=0
run() {  # run <n> <MiB> <dtype> <mem>
  i=$((i+1))
  AKKA_IPC_MEM=$4 timeout -k 10 ${T:-90} python -m torch.distributed.run --nnodes=1 --nproc-per-node=$1 \
    --master-addr 127.0.0.1 --master-port $((29700 + i)) scripts/ipc_open_time.py $2 $3 \
    > gpurun_out/ipc_open/run$i.log 2>&1
  local rc=$?
  grep -E "enable_ipc|windows open|File|Timeout" gpurun_out/ipc_open/run$i.log | head -12
  echo "n=$1 $2MiB $3 $4 rc=$rc"
  return $rc
}
if [ -n "$SPEC" ]; then  # one case: SPEC="<n> <MiB> <dtype> <mem>"
  run $SPEC || exit $?
  exit 0
fi
for spec in "2 384 float32 fine" "2 512 float32 fine" "2 768 float32 fine" "2 1024 float32 fine"; do
  run $spec || exit $?
done
