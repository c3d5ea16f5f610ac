#!/bin/bash
# Round-3 GPU pass AF: bench.py's N-rank flow at N=2, 2 processes sharing the
# card, ipc data plane, every extra, on the final tree (rehearsal, not the metric).
set -o pipefail
mkdir -p gpurun_out/r03af
AKKA_SHARE_GPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29641 bench.py --gpus 2 --data-plane ipc --steps 10 --warmup 3 \
  > gpurun_out/r03af/bench_n2.json 2> gpurun_out/r03af/bench_n2.err
