#!/bin/bash
# Round-4 pass I: the DDP hook tests (tuned lane may be the one-sided lane),
# smoke(), bench.py N=1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r04i
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_dp_ipc_gpu.py -v --timeout 200 --timeout-method thread \
  > $O/pytest_ddp.log 2>&1 || { echo "pytest rc=$?"; tail -40 $O/pytest_ddp.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $O/pytest_ddp.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench_n1.json 2> $O/bench_n1.err || { echo "bench rc=$?"; tail -20 $O/bench_n1.err; exit 1; }
cut -c1-300 $O/bench_n1.json
