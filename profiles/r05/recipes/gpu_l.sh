#!/bin/bash
# Round-5 pass L: kernel traces of the DDP step on the one-sided transport
# (2 ranks on the card): async rounds with the bounded footprint (cu_keep 4)
# and sync rounds with the same mask, to see where the async step's time goes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
O=gpurun_out/r05/l
mkdir -p $O
i=0
for m in async sync; do
  i=$((i+1)); mkdir -p $O/trace_$m
  AKKA_SHARE_GPU=1 GPU_MAX_HW_QUEUES=8 AKKA_OS_DEDICATED=1 AKKA_OS_ROLE_WGS=48 timeout -k 10 150 \
    python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port $((29880+i)) \
    --no-python rocprofv3 --kernel-trace --output-format csv -d $O/trace_$m -o run_%pid% -- python bench/ddp_overlap.py \
    --transport onesided --cu-keep 4 --modes $m --steps 8 --warmup 3 > $O/trace_$m.log 2>&1 \
    || { echo "trace $m rc=$?"; tail -20 $O/trace_$m.log; exit 1; }
  grep ms_per_step $O/trace_$m.log
done
