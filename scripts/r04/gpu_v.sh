#!/bin/bash
# Round-4 pass V: reduce-role workgroups of the one-sided round on the shared
# card (4 ranks, exact): pieces per part follow (AKKA_OS_REDUCE_WGS).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r04v
mkdir -p $O
i=0
for V in 0 64 128 184 256; do
  i=$((i+1)); mkdir -p $O/v$i
  E=""; [ "$V" != "0" ] && E="AKKA_OS_REDUCE_WGS=$V"
  env $E timeout -k 10 200 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=4 \
    --master-addr 127.0.0.1 --master-port $((29810+i)) bench/onesided_round.py --sizes-mb 64,256 --lanes onesided \
    --out-dir $O/v$i > $O/v$i.log 2>&1 || { echo "v$i rc=$?"; tail -20 $O/v$i.log; exit 1; }
  echo "== reduce wgs $V"; python scripts/r04/summarize_round.py $O/v$i 4 | tee $O/v$i.jsonl | cut -c1-230
done
