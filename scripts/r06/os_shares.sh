#!/bin/bash
# Round 6: one-sided exact rounds at N=4 on the card, 256 MiB, window output,
# role shares of the shared-card budget (push,reduce,copy) -- the in-place
# copy role has nothing to copy; ipc_direct as the reference.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06/${1:-os_shares}
mkdir -p $O
port=29841
run() {  # tag, lanes, env...
  port=$((port+1))
  mkdir -p $O/$1
  env "${@:3}" timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node=4 --master-addr 127.0.0.1 \
    --master-port $port bench/onesided_round.py --sizes-mb ${SIZES:-256} --lanes $2 --ipc-lane ipc_fused_lite \
    --steps 20 --warmup 5 --out-dir $O/$1 > $O/$1.log 2>&1 || { echo "$1 rc=$?"; tail -30 $O/$1.log; exit 1; }
  python -c "
import json,glob
rows={}
for f in glob.glob('$O/$1/rank*.json'):
    for c in json.load(open(f))['cases']: rows.setdefault((c['lane'],c['size_mb']),[]).append(c.get('ms'))
for k,v in sorted(rows.items()): print('%-10s %-24s %6g MiB %8.4f ms' % ('$1', k[0], k[1], max(v)))"
}
run direct ipc_direct AKKA_X=0
run wo_121 onesided_wo AKKA_OS_SHARES=1,2,1
run wo_251 onesided_wo AKKA_OS_SHARES=2,5,1
run wo_141 onesided_wo AKKA_OS_SHARES=1,4,1
run wo_231 onesided_wo AKKA_OS_SHARES=2,3,1
run wo_251_b1024 onesided_wo AKKA_OS_SHARES=2,5,1 AKKA_OS_SHARED_BUDGET=1024
