#!/bin/bash
# Round 6: is the small-round gap of r05 (engine path 110 us vs direct 25 us,
# 64 Ki elements, 2 ranks on the card) the lane or its place in the job?
#   same   -- one lane four times in one job (each instance kept alive while
#             the next is created, as bench/small_rounds.py does by default)
#   free   -- the same, each instance freed before the next
#   alone  -- every lane in a job of its own, twice, alternating
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06/${1:-order_ab}
mkdir -p $O
rm -f $O/*.jsonl
port=29651
run() {  # tag, extra args
  port=$((port+1))
  timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 \
    --master-port $port bench/small_rounds.py --mode nk --sizes 65536 --out $O/$1.jsonl "${@:2}" > $O/$1.log 2>&1 \
    || { echo "$1 rc=$?"; tail -20 $O/$1.log; exit 1; }
  echo "== $1"; python -c "
import json,sys
for l in open('$O/$1.jsonl'):
    d=json.loads(l); print('  %-34s host %6.2f wall %7.2f lat %7.2f %s' % (d['lane'], d['host_us_per_call'], d['wall_us_per_call'], d['latency_us'], d.get('windows_id','')))"
}
FOUR=ipc_fused_lite,ipc_fused_lite,ipc_fused_lite,ipc_fused_lite
if [ -n "$QUEUES" ]; then
  # is it the hardware-queue mapping of the streams each instance creates?
  run user_stream --user-stream --lanes $FOUR
  GPU_MAX_HW_QUEUES=8 run hwq8 --lanes $FOUR
  AKKA_COMM_PRIORITY=normal run normal_prio --lanes $FOUR
  exit 0
fi
run same --lanes $FOUR
run free --free --lanes $FOUR
for rep in 1 2; do
  for L in ipc_fused_lite ipc_fused_lite_direct onesided; do run alone_${L}_$rep --lanes $L; done
done
