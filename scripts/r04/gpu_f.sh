#!/bin/bash
# Round-4 pass F: the one-sided lane with the finish folded into the round
# launch (last workgroup out) and distributed zeroing: GPU tests, the cluster
# (actor API) test, a shared-card budget sweep at 256 MiB next to
# ipc_fused_lite, config 4, the reduce role.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r04f
mkdir -p $O/cluster
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_onesided_gpu.py \
  tests/test_graph_step_gpu.py > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
AKKA_TEST_LOGS=$O/cluster timeout -k 10 400 python -u -m pytest -x -v -s --timeout 350 --timeout-method thread \
  tests/test_cluster_onesided_gpu.py > $O/pytest_cluster.log 2>&1 || { echo "cluster rc=$?"; tail -30 $O/pytest_cluster.log; }
tail -3 $O/pytest_cluster.log
port=29640
for B in 512 768 1024; do
  port=$((port+1)); mkdir -p $O/b$B
  AKKA_OS_SHARED_BUDGET=$B timeout -k 10 200 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=4 \
    --master-addr 127.0.0.1 --master-port $port bench/onesided_round.py --sizes-mb 64,256 --lanes onesided,ipc \
    --out-dir $O/b$B > $O/b$B.log 2>&1 || { echo "budget $B rc=$?"; tail -20 $O/b$B.log; exit 1; }
  echo "budget $B"; python scripts/r04/summarize_round.py $O/b$B 4 | tee $O/b$B.jsonl
done
mkdir -p $O/cfg4
timeout -k 10 200 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=4 --master-addr 127.0.0.1 \
  --master-port 29650 bench/onesided_round.py --sizes-mb 64 --lanes onesided --straggler --cfg4-rounds 64 \
  --out-dir $O/cfg4 > $O/cfg4.log 2>&1 || { echo "cfg4 rc=$?"; tail -20 $O/cfg4.log; exit 1; }
python scripts/r04/summarize_round.py $O/cfg4 4 | tee $O/cfg4.jsonl
timeout -k 10 120 python -u bench/onesided_role.py --n 4,8 --threads 256,1024 --grid 256,512 > $O/role.jsonl 2>&1 \
  || { echo "role rc=$?"; tail -20 $O/role.jsonl; exit 1; }
cat $O/role.jsonl
