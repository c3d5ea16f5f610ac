#!/bin/bash
# Round-5 pass D: engine-path table (separate jobs per lane variant), then
# bench.py's N-rank flow with the default (pruned) lane set, 2 and 4 ranks
# sharing the card (ipc data plane; the numbers are HBM-local, not xGMI).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05/d
mkdir -p $O
bash scripts/r05/engine_path.sh engine_path_d > $O/engine_path.txt 2>&1 || { echo "engine path rc=$?"; tail -30 $O/engine_path.txt; exit 1; }
cat $O/engine_path.txt | tail -30
for N in 2 4; do
  AKKA_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node=$N \
    --master-addr 127.0.0.1 --master-port $((29750+N)) bench.py --gpus $N --data-plane ipc --extras off \
    --link-probe off > $O/bench_n$N.json 2> $O/bench_n$N.err || { echo "bench n$N rc=$?"; tail -20 $O/bench_n$N.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_n$N.json')); print($N, d['value'], d['ms_per_step'], d['lane'], json.dumps(d.get('lane_select')))"
done
