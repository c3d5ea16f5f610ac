#!/bin/bash
# Round 6: where the host time of a small exact round goes.
#   n1   -- ThresholdAllreduce at N=1 and its pieces (bench/small_rounds.py)
#   n2   -- 2 ranks on the card: engine-path ipc round vs direct vs one-sided
#   prof -- the n1 64 Ki case under rocprofv3 (kernel + HIP API trace)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06/${1:-small}
mkdir -p $O
rm -f $O/n1.jsonl $O/n2.jsonl
timeout -k 10 300 python -u bench/small_rounds.py --mode n1 --out $O/n1.jsonl > $O/n1.log 2>&1 \
  || { echo "n1 rc=$?"; tail -30 $O/n1.log; exit 1; }
cat $O/n1.jsonl
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 \
  --master-port 29611 bench/small_rounds.py --mode nk --sizes 65536 --out $O/n2.jsonl > $O/n2.log 2>&1 \
  || { echo "n2 rc=$?"; tail -30 $O/n2.log; exit 1; }
cat $O/n2.jsonl
if [ -z "$NOPROF" ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --stats --output-format csv -d $O/prof -o n1 \
  -- python3 bench/small_rounds.py --mode n1 --sizes 65536 --calls 200 > $O/prof.log 2>&1 \
  || { echo "prof rc=$?"; tail -30 $O/prof.log; exit 1; }
ls -R $O/prof | head -20
fi
