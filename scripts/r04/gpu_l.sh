#!/bin/bash
# Round-4 pass L: config 5 at N=2 on the card (ipc data plane; the lane
# selection's choice, whole-step graph variant), with the bench's extras
# watchdog short enough to dump stacks before the box's silence limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r04l
mkdir -p $O
AKKA_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 \
  --master-addr 127.0.0.1 --master-port 29702 bench.py --gpus 2 --data-plane ipc --extras on --extras-only cfg5 \
  --link-probe off --compare-rccl off --steps 4 --warmup 2 --size-mb 16 --extras-deadline-s 100 \
  > $O/bench_n2_cfg5.json 2> $O/bench_n2_cfg5.err || { echo "cfg5 n2 rc=$?"; tail -60 $O/bench_n2_cfg5.err; exit 1; }
tail -12 $O/bench_n2_cfg5.err
python -c "import json; d=json.load(open('$O/bench_n2_cfg5.json')); print(d['lane'], json.dumps(d['extra_configs'])[:1500])"
