#!/bin/bash
# Round-5 pass W: the retracted-marker fix of the overwrite hand-shake on the
# GPU kernel -- the spec harness (every case incl. the new phantom-marker
# replay) and the one-sided GPU tests, then the chaos campaign (pass R).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
O=gpurun_out/r05/w
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_onesided_spec_gpu.py tests/test_onesided_gpu.py tests/test_cluster_onesided_gpu.py > $O/pytest.txt 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/pytest.txt | tail -8
[ $rc -eq 0 ] || exit $rc
bash profiles/r05/recipes/gpu_r.sh
