#!/bin/bash
# ipc lane workgroup size (AKKA_IPC_THREADS) on the shared card: ms per
# 256 MiB fp32 round, pull and bcast, N = 2 and 4 (HBM-local, not xGMI).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ipc_threads
i=0
for n in 2 4; do
  for mode in pull bcast; do
    for t in 256 512 1024; do
      i=$((i+1)); d=gpurun_out/ipc_threads/n${n}_${mode}_t${t}; mkdir -p $d
      AKKA_IPC_THREADS=$t timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node=$n \
        --master-addr 127.0.0.1 --master-port $((29600 + i)) tests/ipc_ranks.py --size 67108864 --rounds 2 \
        --mode $mode --time --out-dir $d > $d/log.txt 2>&1 || { echo "n=$n $mode t=$t failed"; tail -5 $d/log.txt; exit 1; }
      python -c "import json;d=json.load(open('$d/rank0.json'));print('n=$n mode=$mode threads=$t ms/round', round(d['ms_per_round'],3), 'exact', all(d['exact']))"
    done
  done
done
