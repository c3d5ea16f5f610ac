#!/bin/bash
# Counter passes over the kernel microbenchmark.  Each pass is its own
# rocprofv3 run with --kernel-trace only (no sys/runtime traces with --pmc on
# this pool) and holds counters that fit one hardware pass (FETCH_SIZE and
# WRITE_SIZE each expand to many TCC counters: one per pass).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
O=$R/gpurun_out/pmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
ARGS="$R/bench/reduce_kernel_bw.py --sizes-mb 32,256 --nsrc 2,8 --dtypes float32 --iters 5"
i=0
for C in "FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS" "SQ_INSTS_VMEM_RD SQ_WAVES" "MemUnitStalled"; do
  i=$((i+1))
  timeout -k 10 150 rocprofv3 --kernel-trace --pmc $C --output-format csv -d $O/p$i -o run -- python3 $ARGS > $O/p$i.log 2>&1 || { echo "pass $i ($C) rc=$?"; exit 1; }
done
python3 $R/scripts/pmc_summary.py $O/p1 $O/p2 $O/p3 $O/p4 $O/p5 > $O/summary.txt 2>&1
cat $O/summary.txt | head -40
