#!/bin/bash
# ipc lane timing with N processes sharing ONE GPU (HBM-local traffic, not xGMI):
# kernel efficiency of push / reduce / pull, not a link measurement.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ipc_time
for n in 2 4; do
  for pb in 131072 524288 1048576; do
    d=gpurun_out/ipc_time/n${n}_p${pb}
    mkdir -p $d
    AKKA_IPC_PORTION_BYTES=$pb timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node=$n \
      --master-addr 127.0.0.1 --master-port $((29500 + n + pb % 97)) tests/ipc_ranks.py --size 67108864 --rounds 2 \
      --time --out-dir $d > $d/log.txt 2>&1 || { echo "n=$n pb=$pb failed"; tail -5 $d/log.txt; exit 1; }
    echo "n=$n portion=$pb $(cat $d/rank0.json)"
  done
done
