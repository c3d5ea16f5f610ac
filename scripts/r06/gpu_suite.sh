#!/bin/bash
# Round 6: bench.py N=1 (the driver's BENCH run) then the GPU test suite.
# Usage: scripts/r06/gpu_suite.sh <tag> [pytest selection...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06/${1:-suite}
shift
mkdir -p $O
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_n1.json 2> $O/bench_n1.err \
  || { echo "bench rc=$?"; tail -20 $O/bench_n1.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench_n1.json').read().strip().splitlines()[-1])
print({k: d[k] for k in ('value','ms_per_step','host_us_per_round','exact')})"
timeout -k 10 1500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu ${@:-tests} \
  > $O/pytest.txt 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/pytest.txt | tail -8
exit $rc
