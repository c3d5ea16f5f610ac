#!/bin/bash
# Round 6 final tree: bench.py N=1 (the driver's BENCH run), its kernel
# profile, smoke(), then the whole GPU test suite.
# Usage: scripts/r06/final.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06/${1:-final}
mkdir -p $O
timeout -k 10 300 python bench.py > $O/bench_n1.json 2> $O/bench_n1.err \
  || { echo "bench rc=$?"; tail -20 $O/bench_n1.err; exit 1; }
tail -1 $O/bench_n1.json | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench_n1 \
  -- python3 bench.py --steps 20 --warmup 5 > $O/prof.log 2>&1 || { echo "prof rc=$?"; tail -20 $O/prof.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 \
  || { echo "smoke rc=$?"; tail -20 $O/smoke.txt; exit 1; }
cat $O/smoke.txt | tail -2
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest.txt 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/pytest.txt | tail -8
exit $rc
