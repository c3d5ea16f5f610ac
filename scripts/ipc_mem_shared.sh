#!/bin/bash
# ipc lane window memory kind (AKKA_IPC_MEM: fine | uncached | coarse) on a
# shared card: ms per 256 MiB round and exactness, 2 and 4 ranks.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ipc_mem
for mem in coarse fine uncached; do
  for n in 2 4; do
    for mode in pull bcast; do
      d=gpurun_out/ipc_mem/${mem}_n${n}_$mode
      mkdir -p $d
      AKKA_IPC_MEM=$mem timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node=$n \
        --master-addr 127.0.0.1 --master-port $((29300 + n * 11 + ${#mode} + ${#mem} * 3)) tests/ipc_ranks.py \
        --size 67108864 --rounds 3 --time --mode $mode --out-dir $d > $d/log.txt 2>&1 \
        || { echo "$mem n=$n $mode failed"; tail -5 $d/log.txt; exit 1; }
      python -c "import json; d=json.load(open('$d/rank0.json')); print('mem=$mem n=$n mode=$mode', d['ipc']['memory'], d['exact'], d['ipc_error'], round(d['ms_per_round'],3))"
    done
  done
done
