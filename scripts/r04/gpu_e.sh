#!/bin/bash
# Round-4 pass E: one-sided lane round times next to ipc_fused_lite (4
# processes), config 4, the reduce role alone, a per-rank kernel trace; the
# whole-step graph tests; the cluster (actor API) GPU test with logs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r04e
mkdir -p $O/base $O/trace $O/cluster
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=4 --master-addr 127.0.0.1 \
  --master-port 29630 bench/onesided_round.py --sizes-mb 64,256 --straggler --out-dir $O/base \
  > $O/base.log 2>&1 || { echo "base rc=$?"; tail -30 $O/base.log; exit 1; }
python scripts/r04/summarize_round.py $O/base 4 | tee $O/base_summary.jsonl
timeout -k 10 120 python -u bench/onesided_role.py --n 2,4,8 --threads 256,1024 --grid 256,512 > $O/role.jsonl 2>&1 \
  || { echo "role rc=$?"; tail -20 $O/role.jsonl; exit 1; }
cat $O/role.jsonl
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node=4 --master-addr 127.0.0.1 \
  --master-port 29631 --no-python rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run_%pid% \
  -- python bench/onesided_round.py --sizes-mb 64,256 --lanes onesided,ipc --steps 5 --out-dir $O/trace \
  > $O/trace.log 2>&1 || { echo "trace rc=$?"; grep -v "^    @" $O/trace.log | tail -20; exit 1; }
python scripts/r04/ktrace.py $O/trace 8 | tee $O/trace_summary.txt | head -40
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_graph_step_gpu.py \
  > $O/pytest_graph.log 2>&1 || { echo "graph rc=$?"; tail -40 $O/pytest_graph.log; exit 1; }
tail -3 $O/pytest_graph.log
AKKA_TEST_LOGS=$O/cluster timeout -k 10 400 python -u -m pytest -x -v -s --timeout 350 --timeout-method thread \
  tests/test_cluster_onesided_gpu.py > $O/pytest_cluster.log 2>&1 || { echo "cluster rc=$?"; tail -40 $O/pytest_cluster.log; exit 1; }
tail -3 $O/pytest_cluster.log
