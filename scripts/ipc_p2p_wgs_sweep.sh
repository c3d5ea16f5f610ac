#!/bin/bash
# Mailbox p2p (ipc_p2p data plane) workgroups per piece: bench.py's lane
# selection times on 4 processes sharing the card, per AKKA_IPC_P2P_WGS.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/p2p_wgs
i=0
for w in 8 32; do
  i=$((i+1)); o=gpurun_out/p2p_wgs/w$w
  AKKA_SHARE_GPU=1 GPU_MAX_HW_QUEUES=8 AKKA_IPC_P2P_WGS=$w timeout -k 10 240 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node=4 --master-addr 127.0.0.1 --master-port $((29650 + i)) bench.py --gpus 4 --steps 10 --warmup 3 \
    --compare-rccl off --data-plane ipc_p2p --extras off --ipc off > $o.json 2> $o.err || { echo "w=$w failed"; tail -5 $o.err; exit 1; }
  python -c "import json;d=json.load(open('$o.json'));print('wgs=$w', {k:(v['ms'] if isinstance(v,dict) else v) for k,v in d['lane_select'].items()}, 'exact', d['exact'])"
done
