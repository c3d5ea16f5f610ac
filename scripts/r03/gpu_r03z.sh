#!/bin/bash
# Round-3 GPU pass Z: bench.py's N-rank flow, 4 processes sharing the card,
# ipc data plane, every extra (the graphed config-5 step at N>1 for the
# first time) -- a rehearsal of the flow, not the metric.
set -o pipefail
mkdir -p gpurun_out/r03z
AKKA_SHARE_GPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29631 bench.py --gpus 4 --data-plane ipc --steps 10 --warmup 3 \
  > gpurun_out/r03z/bench_n4.json 2> gpurun_out/r03z/bench_n4.err
