#!/bin/bash
# Raw TCC/EA request counters over the chunk-reduce microbenchmark, one
# rocprofv3 pass per hardware counter group (<= 4 TCC counters a pass), plus
# the derived FETCH_SIZE for comparison.  Summary: scripts/pmc_bytes.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
O=$R/gpurun_out/pmc_raw
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
ARGS="$R/bench/reduce_kernel_bw.py --sizes-mb 4,32,256 --nsrc 2,8 --dtypes float32 --impls vec,lds --iters 5"
i=0
for C in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum" \
         "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_DRAM_sum TCC_BUBBLE_sum" \
         "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $C --output-format csv -d $O/p$i -o run -- python3 $ARGS > $O/p$i.log 2>&1 || { echo "pass $i ($C) rc=$?"; tail -5 $O/p$i.log; exit 1; }
done
python3 $R/scripts/pmc_bytes.py $O/p1 $O/p2 $O/p3 > $O/summary.txt 2>&1
cat $O/summary.txt
