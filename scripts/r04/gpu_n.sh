#!/bin/bash
# Round-4 pass N: the one-sided lane on a CU-masked stream when ranks share
# the card: config 5's DP step probe (was: the peer's fp32 GEMMs starved until
# the lane's wait timed out), the one-sided + graph GPU tests, round times at
# 64 / 256 MiB next to ipc_fused_lite, bench config 5 at N=2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r04n
mkdir -p $O/rt
for i in 1 2; do
  AKKA_SHARE_GPU=1 timeout -k 10 120 python -u -m torch.distributed.run --nnodes=1 \
    --nproc-per-node=2 --master-addr 127.0.0.1 --master-port $((29740+i)) bench/os_probe.py --which none \
    --dp-steps 3 --blocks 5,20 --timeout-s 1 > $O/probe_$i.log 2>&1 \
    || { echo "probe $i rc=$?"; grep -v Warning $O/probe_$i.log | tail -30; exit 1; }
  echo "== probe $i"; grep '"dp_step"\|dp_block\|dp_error' $O/probe_$i.log | cut -c1-260
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_onesided_gpu.py \
  tests/test_graph_step_gpu.py > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=4 --master-addr 127.0.0.1 \
  --master-port 29749 bench/onesided_round.py --sizes-mb 64,256 --lanes onesided,ipc --out-dir $O/rt \
  > $O/rt.log 2>&1 || { echo "rt rc=$?"; tail -20 $O/rt.log; exit 1; }
python scripts/r04/summarize_round.py $O/rt 4 | tee $O/rt.jsonl | cut -c1-330
AKKA_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 \
  --master-addr 127.0.0.1 --master-port 29748 bench.py --gpus 2 --data-plane ipc --extras on --extras-only cfg5 \
  --link-probe off --compare-rccl off --steps 4 --warmup 2 --size-mb 16 --extras-deadline-s 150 \
  > $O/bench_n2_cfg5.json 2> $O/bench_n2_cfg5.err || { echo "cfg5 n2 rc=$?"; tail -40 $O/bench_n2_cfg5.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_n2_cfg5.json')); print(d['lane'], json.dumps(d.get('extra_configs'))[:1500], d.get('extras_error'))"
