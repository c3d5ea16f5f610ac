#!/bin/bash
# Round-5 pass O: the one-sided push with 128 B per thread per batch (half the
# write-through ack waits per part): role timeline (window output), the lane
# table vs the direct ipc round, bench.py's N=4 / N=2 selection, 4 / 2 ranks
# on the card; then the one-sided GPU tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
O=gpurun_out/r05/o
mkdir -p $O/wo $O/time_wo $O/time_direct
timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node=4 --master-addr 127.0.0.1 \
  --master-port 29941 bench/onesided_timeline.py --window-output --out-dir $O/wo > $O/wo.log 2>&1 || { echo "wo rc=$?"; tail -20 $O/wo.log; exit 1; }
for V in wo:onesided_wo direct:ipc_direct; do
  T=${V%%:*}; L=${V#*:}
  timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node=4 --master-addr 127.0.0.1 \
    --master-port $((29942+${#T})) bench/onesided_round.py --sizes-mb 64,256 --lanes $L --ipc-lane ipc_fused_lite \
    --steps 20 --warmup 5 --out-dir $O/time_$T > $O/time_$T.log 2>&1 || { echo "time $T rc=$?"; tail -30 $O/time_$T.log; exit 1; }
  echo "== $T"; grep "rank 0:" $O/time_$T.log | cut -c1-160
done
for N in 4 2; do
  AKKA_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node=$N \
    --master-addr 127.0.0.1 --master-port $((29950+N)) bench.py --gpus $N --data-plane ipc --extras off \
    --link-probe off > $O/bench_n$N.json 2> $O/bench_n$N.err || { echo "bench n$N rc=$?"; tail -20 $O/bench_n$N.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_n$N.json')); print($N, d['value'], d['ms_per_step'], d['lane'], json.dumps(d.get('lane_select')))"
done
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_onesided_gpu.py > $O/pytest.txt 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/pytest.txt | tail -8
exit $rc
