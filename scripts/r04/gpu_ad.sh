#!/bin/bash
# Round-4 pass AD: bench.py's headline flow at N=2 and N=4 on one card (ipc
# data plane, extras off): the lane selection's final-tree picks.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r04ad
mkdir -p $O
for N in 2 4; do
  AKKA_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node=$N \
    --master-addr 127.0.0.1 --master-port $((29850+N)) bench.py --gpus $N --data-plane ipc --extras off \
    --link-probe off > $O/bench_n$N.json 2> $O/bench_n$N.err || { echo "bench n$N rc=$?"; tail -20 $O/bench_n$N.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_n$N.json')); print($N, d['value'], d['ms_per_step'], d['lane'], json.dumps(d.get('checks')), json.dumps({k: v.get('ms') for k, v in d['lane_select'].items() if isinstance(v, dict)}))"
done
