#!/bin/bash
# Round-4 pass B: the restructured one-sided lane (one role-partitioned
# launch + finish).  GPU tests of the lane, whole-round times next to
# ipc_fused_lite (4 processes on the card), config 4, the reduce role alone,
# and a per-rank kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r04b
mkdir -p $O/base $O/trace
timeout -k 10 700 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_onesided_gpu.py \
  tests/test_cluster_onesided_gpu.py tests/test_graph_step_gpu.py \
  > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=4 --master-addr 127.0.0.1 \
  --master-port 29620 bench/onesided_round.py --sizes-mb 64,256 --straggler --out-dir $O/base \
  > $O/base.log 2>&1 || { echo "base rc=$?"; tail -30 $O/base.log; exit 1; }
python scripts/r04/summarize_round.py $O/base 4
timeout -k 10 120 python -u bench/onesided_role.py --n 2,4,8 --threads 256,1024 --grid 256,512 > $O/role.jsonl 2>&1 \
  || { echo "role rc=$?"; tail -20 $O/role.jsonl; exit 1; }
cat $O/role.jsonl
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node=4 --master-addr 127.0.0.1 \
  --master-port 29621 --no-python rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run_%pid% \
  -- python bench/onesided_round.py --sizes-mb 64,256 --lanes onesided --steps 5 --out-dir $O/trace \
  > $O/trace.log 2>&1 || { echo "trace rc=$?"; grep -v "^    @" $O/trace.log | tail -20; exit 1; }
ls $O/trace
for f in $(find $O/trace -name "*kernel_stats.csv" | head -1); do head -8 "$f" | cut -c1-220; done
