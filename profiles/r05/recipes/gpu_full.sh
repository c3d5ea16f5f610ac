#!/bin/bash
# Round-5: the whole GPU suite (what the driver runs at round end) + smoke().
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
O=gpurun_out/r05/full
mkdir -p $O
timeout -k 10 1100 python -u -m pytest -v --timeout 240 --timeout-method thread -m gpu tests/ > $O/pytest.txt 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/pytest.txt | tail -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1; rc=$?
tail -3 $O/smoke.txt
exit $rc
