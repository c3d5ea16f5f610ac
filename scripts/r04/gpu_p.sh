#!/bin/bash
# Round-4 pass P: CU mask opt-in (cu_keep): DP probe with and without it,
# bench config 5 at N=2 (opts in on a shared card), round times without it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r04p
mkdir -p $O/rt
for K in 6 0; do
  AKKA_SHARE_GPU=1 timeout -k 10 120 python -u -m torch.distributed.run --nnodes=1 \
    --nproc-per-node=2 --master-addr 127.0.0.1 --master-port $((29760+K)) bench/os_probe.py --which none \
    --dp-steps 2 --blocks 5,20 --timeout-s 1 --cu-keep $K > $O/probe_k$K.log 2>&1 \
    || { echo "probe $K rc=$?"; grep -v Warning $O/probe_k$K.log | tail -30; exit 1; }
  echo "== cu_keep $K"; grep 'dp_block\|dp_error' $O/probe_k$K.log | cut -c1-200
done
AKKA_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 \
  --master-addr 127.0.0.1 --master-port 29768 bench.py --gpus 2 --data-plane ipc --extras on --extras-only cfg5 \
  --link-probe off --compare-rccl off --steps 4 --warmup 2 --size-mb 16 --extras-deadline-s 150 \
  > $O/bench_n2_cfg5.json 2> $O/bench_n2_cfg5.err || { echo "cfg5 n2 rc=$?"; tail -40 $O/bench_n2_cfg5.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_n2_cfg5.json')); print(d['lane'], json.dumps(d.get('extra_configs'))[:1500], d.get('extras_error'))"
timeout -k 10 200 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=4 --master-addr 127.0.0.1 \
  --master-port 29769 bench/onesided_round.py --sizes-mb 64,256 --lanes onesided,ipc --out-dir $O/rt \
  > $O/rt.log 2>&1 || { echo "rt rc=$?"; tail -20 $O/rt.log; exit 1; }
python scripts/r04/summarize_round.py $O/rt 4 | tee $O/rt.jsonl | cut -c1-200
timeout -k 10 400 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_onesided_gpu.py \
  tests/test_graph_step_gpu.py tests/test_dp_ipc_gpu.py > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
