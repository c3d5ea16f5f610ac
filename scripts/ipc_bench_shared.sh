#!/bin/bash
# bench.py's N-rank flow on ONE GPU: N processes share the card, ipc-only data
# plane (no RCCL communicator can hold two ranks of one GPU).  Numbers are
# HBM-local, not xGMI: a rehearsal of the multi-rank bench path.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/bench_shared
for n in 2 4; do
  AKKA_SHARE_GPU=1 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node=$n \
    --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --gpus $n --steps 20 --warmup 5 \
    --data-plane ipc --compare-rccl off --extras off > gpurun_out/bench_shared/n$n.json \
    2> gpurun_out/bench_shared/n$n.err || { echo "n=$n rc=$?"; tail -20 gpurun_out/bench_shared/n$n.err; exit 1; }
  cat gpurun_out/bench_shared/n$n.json
done
