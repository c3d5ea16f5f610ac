#!/bin/bash
# Round-4 pass U: shared-card role shares (push, reduce, copy) of the
# one-sided round, 4 ranks, exact, 64 / 256 MiB.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r04u
mkdir -p $O
i=0
for V in "1,2,1" "2,2,1" "3,2,1" "2,3,1" "3,3,1" "2,2,2" "4,3,1"; do
  i=$((i+1)); mkdir -p $O/v$i
  LANES=onesided; [ $i -eq 1 ] && LANES=onesided,ipc
  AKKA_OS_SHARES=$V timeout -k 10 200 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=4 \
    --master-addr 127.0.0.1 --master-port $((29800+i)) bench/onesided_round.py --sizes-mb 64,256 --lanes $LANES \
    --out-dir $O/v$i > $O/v$i.log 2>&1 || { echo "v$i rc=$?"; tail -20 $O/v$i.log; exit 1; }
  echo "== shares $V"; python scripts/r04/summarize_round.py $O/v$i 4 | tee $O/v$i.jsonl | cut -c1-175
done
