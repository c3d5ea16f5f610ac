#!/bin/bash
# Round 6: per-role timeline of a small one-sided exact round (64 Ki fp32,
# 2 ranks on the card): where its ~37 us go (bench/onesided_timeline.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06/${1:-os_small_tl}
mkdir -p $O/tl
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 \
  --master-port 29861 bench/onesided_timeline.py --sizes-mb 0.25 --chunk-mb 4 --calls 20 --out-dir $O/tl \
  > $O/tl.log 2>&1 || { echo "tl rc=$?"; tail -30 $O/tl.log; exit 1; }
grep '"rank"' $O/tl.log
