#!/bin/bash
# Rehearse bench.py's N>1 RCCL path with 2 ranks sharing one GPU (1-GPU box).
# RCCL may refuse two ranks on one device; the log says which way it went.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/sharedgpu
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 AKKA_SHARE_GPU=1 NCCL_DEBUG=WARN
timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 \
  --compare-rccl off --extras off --watchdog-s 120 > $O/n2.json 2> $O/n2.err
rc=$?
echo "rc=$rc"
cat $O/n2.json
tail -25 $O/n2.err
exit $rc
