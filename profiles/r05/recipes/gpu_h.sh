#!/bin/bash
# Round-5 pass H: torch DDP step with the threshold comm hook, 2 ranks on the
# card, sync vs async bucket rounds, per lane (bench/ddp_overlap.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
O=gpurun_out/r05/h
mkdir -p $O
i=0
run() {  # tag, args...
  i=$((i+1)); tag=$1; shift
  AKKA_SHARE_GPU=1 GPU_MAX_HW_QUEUES=8 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 \
    --master-addr 127.0.0.1 --master-port $((29850+i)) bench/ddp_overlap.py "$@" > $O/$tag.log 2>&1 \
    || { echo "$tag rc=$?"; tail -20 $O/$tag.log; return 1; }
  grep ms_per_step $O/$tag.log
}
for m in sync async; do
  run stream_ipc_$m --transport stream --data-plane ipc --modes $m && \
  run stream_ipc_fused_lite_$m --transport stream --data-plane ipc --lane ipc_fused_lite --modes $m && \
  run stream_ipc_fused_lite_direct_$m --transport stream --data-plane ipc --lane ipc_fused_lite_direct --modes $m && \
  run onesided_$m --transport onesided --cu-keep 6 --modes $m || exit 1
done
