#!/bin/bash
# Round-5 pass S: DDP step on the one-sided transport with and without window
# output (exact rounds return the window row; the hook's mean reads it into
# the bucket), bucket views on, 2 ranks on the card, same-box A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
O=gpurun_out/r05/s
mkdir -p $O
i=0
for wo in 0 1 0 1; do
  i=$((i+1))
  AKKA_SHARE_GPU=1 GPU_MAX_HW_QUEUES=8 timeout -k 10 150 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node=2 --master-addr 127.0.0.1 --master-port $((30100+i)) bench/ddp_overlap.py --transport onesided \
    --cu-keep 0 --modes sync --window-output $wo > $O/wo${wo}_$i.log 2>&1 || { echo "wo$wo rc=$?"; tail -20 $O/wo${wo}_$i.log; exit 1; }
  echo "wo$wo $(grep ms_per_step $O/wo${wo}_$i.log)"
done
