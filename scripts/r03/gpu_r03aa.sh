#!/bin/bash
# Round-3 GPU pass AA: cfg3 alone after the headline (no link probe, no cfg4),
# extras sharing the headline's transport: 4 processes sharing the card.
set -o pipefail
mkdir -p gpurun_out/r03aa
AKKA_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29633 bench.py --gpus 4 --data-plane ipc --steps 10 --warmup 3 \
  --extras-only cfg3 --link-probe off > gpurun_out/r03aa/cfg3_only.json 2> gpurun_out/r03aa/cfg3_only.err
