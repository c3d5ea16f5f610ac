#!/bin/bash
# Round-3 GPU pass X: counters of the config-5 graphed step's kernels (fused
# average + SGD + bf16 shadow, column sum, cross entropy): bytes each moves
# (FETCH_SIZE / WRITE_SIZE, one counter pass each) and LDS bank conflicts.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r03x
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for C in "FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C --output-format csv -d $O/p$i -o run -- \
    python3 $R/bench/cfg5_step.py --dtype bf16 --graph --steps 10 --warmup 3 > $O/p$i.log 2>&1 || { echo "pass $i ($C) rc=$?"; exit 1; }
done
python3 $R/scripts/pmc_summary.py $O/p1 $O/p2 $O/p3 > $O/summary.txt 2>&1
