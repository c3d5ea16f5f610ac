#!/bin/bash
# Round-4 pass O: one-sided round times with 4 ranks on the card, by CU mask:
# none (AKKA_OS_CU_MASK=0), 6 / 7 of every 8 CUs; ipc_fused_lite alongside.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r04o
mkdir -p $O
i=0
for V in "AKKA_OS_CU_MASK=0" "AKKA_OS_CU_KEEP=6" "AKKA_OS_CU_KEEP=7" "AKKA_OS_CU_KEEP=7 AKKA_OS_SHARED_BUDGET=768"; do
  i=$((i+1)); mkdir -p $O/v$i
  env $V timeout -k 10 200 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=4 --master-addr 127.0.0.1 \
    --master-port $((29750+i)) bench/onesided_round.py --sizes-mb 64,256 --lanes onesided,ipc --out-dir $O/v$i \
    > $O/v$i.log 2>&1 || { echo "v$i rc=$?"; tail -20 $O/v$i.log; exit 1; }
  echo "== $V"; python scripts/r04/summarize_round.py $O/v$i 4 | tee $O/v$i.jsonl | cut -c1-200
done
