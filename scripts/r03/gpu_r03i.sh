#!/bin/bash
# Round-3 GPU pass I: why bench.py's cfg3 (1 GiB bf16) ran 28.5 ms per round
# at N=4 on the shared card when the same lane alone takes 3.2 ms
# (pass H): cfg3 alone, then the full flow again, now with cfg3's lane and
# ipc mode in the line.
set -o pipefail
mkdir -p gpurun_out/r03i
AKKA_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 4 --data-plane ipc --steps 10 --warmup 3 \
  --extras-only cfg3 --link-probe off > gpurun_out/r03i/bench_cfg3_only.json 2> gpurun_out/r03i/bench_cfg3_only.err &&
AKKA_SHARE_GPU=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29614 bench.py --gpus 4 --data-plane ipc --steps 10 --warmup 3 \
  > gpurun_out/r03i/bench_full.json 2> gpurun_out/r03i/bench_full.err
