#!/bin/bash
# Round-5 pass J (variant wo_new measured a change reverted afterwards, see
# profiles/r05/copy_share/README.md): the one-sided lane with window output on one card (4
# processes, 64/256 MiB fp32): copy role shrunk and its share of the shared
# budget given to push and reduce (default) vs the round-4 shares
# (AKKA_OS_SHARES=1,2,1), the direct ipc round for scale; then bench.py's own
# N=4 and N=2 selection with the default lane set.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
O=gpurun_out/r05/j
mkdir -p $O
port=29721
for V in wo_new:onesided_wo: wo_old:onesided_wo:1,2,1 direct:ipc_direct: ; do
  T=${V%%:*}; R=${V#*:}; L=${R%%:*}; SH=${R#*:}; mkdir -p $O/time_$T
  port=$((port+1))
  AKKA_OS_SHARES=$SH timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node=4 \
    --master-addr 127.0.0.1 --master-port $port bench/onesided_round.py --sizes-mb 64,256 --lanes $L \
    --ipc-lane ipc_fused_lite --steps 20 --warmup 5 --out-dir $O/time_$T > $O/time_$T.log 2>&1 \
    || { echo "time $T rc=$?"; tail -30 $O/time_$T.log; exit 1; }
  echo "== $T"; grep "rank 0:" $O/time_$T.log | cut -c1-300
done
for N in 4 2; do
  AKKA_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node=$N \
    --master-addr 127.0.0.1 --master-port $((29790+N)) bench.py --gpus $N --data-plane ipc --extras off \
    --link-probe off > $O/bench_n$N.json 2> $O/bench_n$N.err || { echo "bench n$N rc=$?"; tail -20 $O/bench_n$N.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_n$N.json')); print($N, d['value'], d['ms_per_step'], d['lane'], json.dumps(d.get('lane_select')))"
done
