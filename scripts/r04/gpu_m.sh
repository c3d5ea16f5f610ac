#!/bin/bash
# Round-4 pass M4: config 5's DP step on the one-sided lane, N=2 on the card,
# full lane stats per step (which gate drops the pushes that never land).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r04m4
mkdir -p $O
for i in 1 2 3; do
  AKKA_SHARE_GPU=1 timeout -k 10 120 python -u -m torch.distributed.run --nnodes=1 \
    --nproc-per-node=2 --master-addr 127.0.0.1 --master-port $((29730+i)) bench/os_probe.py --which none \
    --dp-steps 3 --blocks "" --timeout-s 1 > $O/probe_$i.log 2>&1 \
    || { echo "probe $i rc=$?"; grep -v Warning $O/probe_$i.log | tail -30; exit 1; }
  echo "== $i"; grep '"dp_step"\|dp_error' $O/probe_$i.log | cut -c1-900
done
