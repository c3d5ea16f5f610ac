#!/bin/bash
# Round-4 pass J: bench.py's N-rank flow with 8 processes on the card (ipc
# data plane; lane selection includes the one-sided lane at N=8), then the
# config-4 extra at N=8 (0.75/0.75: the straggler's block is not required).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r04j
mkdir -p $O
AKKA_SHARE_GPU=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node=8 \
  --master-addr 127.0.0.1 --master-port 29690 bench.py --gpus 8 --data-plane ipc --extras off --link-probe off \
  --steps 6 --warmup 2 > $O/bench_n8_shared.json 2> $O/bench_n8_shared.err \
  || { echo "bench n8 rc=$?"; tail -30 $O/bench_n8_shared.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_n8_shared.json')); print(d['value'], d['lane'], json.dumps(d.get('lane_select'))[:1200])"
AKKA_SHARE_GPU=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node=8 \
  --master-addr 127.0.0.1 --master-port 29691 bench.py --gpus 8 --data-plane ipc --extras on --extras-only cfg4 \
  --link-probe off --steps 2 --warmup 1 --size-mb 16 > $O/bench_n8_cfg4.json 2> $O/bench_n8_cfg4.err \
  || { echo "cfg4 n8 rc=$?"; tail -30 $O/bench_n8_cfg4.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_n8_cfg4.json')); print(json.dumps(d['extra_configs'])[:1500])"
