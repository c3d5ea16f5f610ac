#!/bin/bash
# Round-3 GPU pass AB: does cfg3's shared-card slowdown depend on how many
# rounds the headline ran first?  Headline with lane selection off, 1 timed
# step, no warm-up, then cfg3 on the default fenced ipc lane (compare pass K:
# 29.4 ms with 10 steps + 3 warm-up and no transport sharing).
set -o pipefail
mkdir -p gpurun_out/r03ab
AKKA_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29635 bench.py --gpus 4 --data-plane ipc --steps 1 --warmup 0 \
  --extras-only cfg3 --link-probe off --lane-select off --compare-rccl off \
  > gpurun_out/r03ab/cfg3_min.json 2> gpurun_out/r03ab/cfg3_min.err
