#!/bin/bash
# Per-kernel times of the ipc lane (push / reduce / phase 2), 2 ranks sharing
# the card, each rank under its own rocprofv3 (torchrun --no-python starts the
# profiler, which starts python: no exec from a process that touched the GPU).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/ipc_prof
mkdir -p $O
for mode in pull bcast; do
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 \
    --master-port $((29800 + ${#mode})) --no-python rocprofv3 --kernel-trace --stats -d $O/$mode -o run \
    -- python tests/ipc_ranks.py --size 67108864 --rounds 2 --time --mode $mode --out-dir $O \
    > $O/$mode.log 2>&1 || { echo "$mode failed"; tail -20 $O/$mode.log; exit 1; }
  echo "== $mode"; cat $O/rank0.json; echo
  find $O/$mode -name "*kernel_stats.csv" | head -2 | while read f; do echo "-- $f"; head -8 "$f" | cut -c1-220; done
done
