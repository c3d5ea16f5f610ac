#!/bin/bash
# bench.py's N-rank flow on ONE GPU: N processes share the card, no RCCL
# communicator (RCCL refuses two ranks of one device):
#   --data-plane ipc      every exact round on the one-sided lane (pull / bcast)
#   --data-plane ipc_p2p  the p2p schedules over mailboxes + the ipc lanes,
#                         lane selection over all of them, extras incl. cfg4
# Numbers are HBM-local, not xGMI: a rehearsal of the multi-rank bench path.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/bench_shared
run() {  # run <n> <tag> <extra args...>
  local n=$1 tag=$2; shift 2
  AKKA_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=$n \
    --master-addr 127.0.0.1 --master-port $((29600 + n + ${#tag})) bench.py --gpus $n --steps 20 --warmup 5 \
    --compare-rccl off "$@" > gpurun_out/bench_shared/$tag.json 2> gpurun_out/bench_shared/$tag.err \
    || { echo "$tag rc=$?"; tail -20 gpurun_out/bench_shared/$tag.err; return 1; }
  cat gpurun_out/bench_shared/$tag.json
}
STEPS="${STEPS:-ipc2 ipc4 p2p4}"
for s in $STEPS; do
  case $s in
    ipc2) run 2 n2 --data-plane ipc --extras off || exit 1 ;;
    ipc4) run 4 n4 --data-plane ipc --extras off || exit 1 ;;
    ipc8) run 8 n8 --data-plane ipc --extras off || exit 1 ;;
    # 8 processes x 4 hardware queues oversubscribe the card's queue slots
    # (the scheduler then time-slices queues); fewer queues per process:
    ipc8q2) GPU_MAX_HW_QUEUES=2 run 8 n8_q2 --data-plane ipc --extras off || exit 1 ;;
    ipc8q1) GPU_MAX_HW_QUEUES=1 run 8 n8_q1 --data-plane ipc --extras off || exit 1 ;;
    ipc6) run 6 n6 --data-plane ipc --extras off || exit 1 ;;
    ipc7) run 7 n7 --data-plane ipc --extras off || exit 1 ;;
    p2p8) GPU_MAX_HW_QUEUES=4 run 8 p2p_n8 --data-plane ipc_p2p --extras on --extras-only cfg4 \
            --cfg4-size-mb 64 --cfg4-delay-ms 50 --cfg4-rounds 6 || exit 1 ;;
    all4) GPU_MAX_HW_QUEUES=8 run 4 all_n4 --data-plane ipc_p2p --extras on --extras-deadline-s 150 \
            --cfg4-size-mb 64 --cfg4-delay-ms 50 --cfg4-rounds 10 || exit 1 ;;
    p2p4) GPU_MAX_HW_QUEUES=8 run 4 p2p_n4 --data-plane ipc_p2p --extras on --extras-only cfg4,cfg5 \
            --cfg4-size-mb 64 --cfg4-delay-ms 50 --cfg4-rounds 10 || exit 1 ;;
  esac
done
