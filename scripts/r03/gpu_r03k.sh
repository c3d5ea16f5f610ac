#!/bin/bash
# Round-3 GPU pass K: bisect bench.py's slow cfg3 (N=4, shared card, ipc):
# without lane selection (cfg3 on the default fenced ipc lane).
set -o pipefail
mkdir -p gpurun_out/r03k
AKKA_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29615 bench.py --gpus 4 --data-plane ipc --steps 10 --warmup 3 \
  --extras-only cfg3 --link-probe off --lane-select off > gpurun_out/r03k/cfg3_noselect.json 2> gpurun_out/r03k/cfg3_noselect.err
