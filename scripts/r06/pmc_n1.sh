#!/bin/bash
# Round 6: HBM bytes of the N=1 headline round (bench.py, 256 MiB fp32), one
# counter per pass (FETCH_SIZE and WRITE_SIZE do not fit one pass's 4 TCC
# counters), --extras off so only the headline's kernels run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06/${1:-pmc_n1}
mkdir -p $O
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $C --output-format csv -d $O/$C -o n1 \
    -- python3 bench.py --steps 10 --warmup 2 --extras off > $O/$C.log 2>&1 || { echo "pmc $C rc=$?"; tail -20 $O/$C.log; exit 1; }
done
python scripts/pmc_summary.py $O/FETCH_SIZE $O/WRITE_SIZE > $O/summary.txt && cat $O/summary.txt

