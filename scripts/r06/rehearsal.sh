#!/bin/bash
# Round 6 rehearsal: bench.py's whole N-rank flow with every extra config, 8 and
# 4 processes sharing the card (mailbox p2p data plane standing in for RCCL,
# which cannot form a communicator of ranks on one device): a rehearsal of
# the driver's SCALE run with the round-6 default lane set (8 lanes, validation burst).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06/${1:-rehearsal}
mkdir -p $O
for N in 8 4; do
  AKKA_SHARE_GPU=1 timeout -k 10 560 python -m torch.distributed.run --nnodes=1 --nproc-per-node=$N \
    --master-addr 127.0.0.1 --master-port $((29900+N)) bench.py --gpus $N --data-plane ipc_p2p --extras on \
    --extras-deadline-s 400 > $O/bench_n$N.json 2> $O/bench_n$N.err || { echo "bench n$N rc=$?"; tail -30 $O/bench_n$N.err; exit 1; }
  python - <<PY
import json
d = json.load(open("$O/bench_n$N.json"))
print($N, d["value"], d["ms_per_step"], d["lane"], d.get("extras_error"), d.get("checks"))
print(json.dumps(d.get("lane_select"))[:600])
ex = d.get("extra_configs") or {}
for k, v in ex.items():
    print(k, json.dumps(v)[:500])
PY
done
