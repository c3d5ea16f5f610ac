#!/bin/bash
# Round-4 pass K: small-buffer latency of the one-sided round vs the ipc lane
# (4 processes on the card, exact rounds), 64 KiB .. 16 MiB.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r04k
mkdir -p $O/lat
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=4 --master-addr 127.0.0.1 \
  --master-port 29700 bench/onesided_round.py --sizes-mb 0.0625,1,4,16 --chunk-mb 1 --lanes onesided,ipc \
  --steps 50 --warmup 10 --out-dir $O/lat > $O/lat.log 2>&1 || { echo "lat rc=$?"; tail -20 $O/lat.log; exit 1; }
python scripts/r04/summarize_round.py $O/lat 4 | tee $O/lat.jsonl | cut -c1-330
timeout -k 10 600 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_onesided_gpu.py -k chaos \
  > $O/pytest_chaos.log 2>&1 || { echo "chaos rc=$?"; tail -30 $O/pytest_chaos.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $O/pytest_chaos.log
AKKA_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 \
  --master-addr 127.0.0.1 --master-port 29702 bench.py --gpus 2 --data-plane ipc --extras on --extras-only cfg5 \
  --link-probe off --steps 4 --warmup 2 --size-mb 16 > $O/bench_n2_cfg5.json 2> $O/bench_n2_cfg5.err \
  || { echo "cfg5 n2 rc=$?"; tail -30 $O/bench_n2_cfg5.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_n2_cfg5.json')); print(d['lane'], json.dumps(d['extra_configs'])[:1500])"
