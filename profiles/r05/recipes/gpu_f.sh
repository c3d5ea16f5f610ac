#!/bin/bash
# Round-5 pass F: window output of the one-sided lane (no gather copy):
# GPU tests, the lane table (onesided vs onesided_wo vs ipc direct), bench.py
# N=2/4 on one card with the default lane set, TCC write bytes per rank.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
O=gpurun_out/r05/f
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_onesided_gpu.py -k "window_output or exact_rounds" > $O/pytest.txt 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/pytest.txt | tail -10
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|assert" $O/pytest.txt | head -60; exit $rc; }
LANES="onesided onesided_wo ipc_direct" bash profiles/r05/recipes/engine_path.sh wo_table > $O/wo_table.txt 2>&1 || { echo "table rc=$?"; tail -30 $O/wo_table.txt; exit 1; }
tail -12 $O/wo_table.txt
for N in 2 4; do
  AKKA_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node=$N \
    --master-addr 127.0.0.1 --master-port $((29760+N)) bench.py --gpus $N --data-plane ipc --extras off \
    --link-probe off > $O/bench_n$N.json 2> $O/bench_n$N.err || { echo "bench n$N rc=$?"; tail -20 $O/bench_n$N.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_n$N.json')); print($N, d['value'], d['ms_per_step'], d['lane'], d['config']['output'][:40], json.dumps(d.get('lane_select')))"
done
