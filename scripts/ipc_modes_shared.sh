#!/bin/bash
# ipc lane variants on a shared card: ms per 256 MiB round, 2 and 4 ranks.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ipc_modes
for n in 2 4; do
  for mode in pull bcast fused fused_bcast; do
    d=gpurun_out/ipc_modes/n${n}_$mode
    mkdir -p $d
    timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node=$n --master-addr 127.0.0.1 \
      --master-port $((29900 + n * 7 + ${#mode})) tests/ipc_ranks.py --size 67108864 --rounds 2 --time \
      --mode $mode --out-dir $d > $d/log.txt 2>&1 || { echo "n=$n $mode failed"; tail -5 $d/log.txt; exit 1; }
    python -c "import json,sys; d=json.load(open('$d/rank0.json')); print('n=$n mode=$mode', d['exact'], d['ipc_error'], round(d['ms_per_round'],3))"
  done
done
