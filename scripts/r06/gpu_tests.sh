#!/bin/bash
# Round 6: a pytest -m gpu selection, verbose, one process.
# Usage: scripts/r06/gpu_tests.sh <tag> <pytest paths / -k ...>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06/${1:-tests}
shift
mkdir -p $O
timeout -k 10 1100 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu "$@" > $O/pytest.txt 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/pytest.txt | tail -8
exit $rc
