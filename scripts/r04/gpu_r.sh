#!/bin/bash
# Round-4 pass R: bench.py's full N-rank flow with every extra config, 4
# processes on the card (ipc data plane; the driver's node runs the rccl
# plane on 4 GPUs) -- a rehearsal of the SCALE run's N=4 point.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r04r
mkdir -p $O
AKKA_SHARE_GPU=1 timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node=4 \
  --master-addr 127.0.0.1 --master-port 29780 bench.py --gpus 4 --data-plane ipc --extras on \
  > $O/bench_n4_all.json 2> $O/bench_n4_all.err || { echo "bench rc=$?"; tail -40 $O/bench_n4_all.err; exit 1; }
grep "phase\|extra" $O/bench_n4_all.err | tail -20
python -c "import json; d=json.load(open('$O/bench_n4_all.json')); print(d['value'], d['lane'], d.get('extras_error')); print(json.dumps(d['extra_configs'])[:3000])"
