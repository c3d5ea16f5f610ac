#!/bin/bash
# Round 6: the small-round table of profiles/r06/small_rounds/README.md on
# the final tree.
#   n1     -- ThresholdAllreduce at N=1: host / wall us per call and its pieces
#   n2     -- 2 ranks on the card, 64 Ki elements, every lane in one job on the
#             caller's own stream (--user-stream: no shared-card queue state
#             between the instances), twice
#   prof   -- the n1 64 Ki case under rocprofv3 --kernel-trace --stats
#   tl     -- one-sided N=4 256 MiB per-role timeline (window output), and the
#             same with every rank on 2 of each 8 CUs (cu_keep)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06/${1:-small_final}
mkdir -p $O
rm -f $O/*.jsonl
timeout -k 10 300 python -u bench/small_rounds.py --mode n1 --out $O/n1.jsonl > $O/n1.log 2>&1 \
  || { echo "n1 rc=$?"; tail -30 $O/n1.log; exit 1; }
cat $O/n1.jsonl
port=29671
for rep in 1 2; do
  port=$((port+1))
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 \
    --master-port $port bench/small_rounds.py --mode nk --sizes 65536 --user-stream \
    --lanes ipc_fused_lite,ipc_fused_lite_direct,onesided --out $O/n2_$rep.jsonl > $O/n2_$rep.log 2>&1 \
    || { echo "n2 rc=$?"; tail -30 $O/n2_$rep.log; exit 1; }
  cat $O/n2_$rep.jsonl
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o n1 \
  -- python3 bench/small_rounds.py --mode n1 --sizes 65536 --calls 200 > $O/prof.log 2>&1 \
  || { echo "prof rc=$?"; tail -30 $O/prof.log; exit 1; }
for K in 0 2; do
  port=$((port+1))
  mkdir -p $O/tl_keep$K
  AKKA_OS_CU_DISJOINT=1 AKKA_OS_CU_KEEP=$K timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=4 \
    --master-addr 127.0.0.1 --master-port $port bench/onesided_timeline.py --sizes-mb 256 --window-output \
    --out-dir $O/tl_keep$K > $O/tl_keep$K.log 2>&1 || { echo "tl $K rc=$?"; tail -30 $O/tl_keep$K.log; exit 1; }
  grep '"rank"' $O/tl_keep$K.log | head -4
done
