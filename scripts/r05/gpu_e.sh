#!/bin/bash
# Round-5 pass E: the reference spec's arrival orders on the real round
# kernel (tests/test_onesided_spec_gpu.py), then bench.py N=1 (regression
# check of the engine-path changes on the local round).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05/e
mkdir -p $O
# (clock_probe.py: lane timeouts match the wall clock, 510 / 2006 ms for 500 / 2000 ms)
timeout -k 10 60 python scripts/r05/nowait_probe.py && timeout -k 10 900 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu \
  tests/test_onesided_spec_gpu.py > $O/pytest.txt 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest.txt | tail -40
[ $rc -eq 0 ] || { grep -B5 -A40 "Error\|assert" $O/pytest.txt | head -80; exit $rc; }
timeout -k 10 300 python bench.py > $O/bench_n1.json 2> $O/bench_n1.err || { echo "bench n1 rc=$?"; tail -20 $O/bench_n1.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_n1.json')); print(d['value'], d['ms_per_step'], {k: v for k, v in d.get('extra_configs', {}).items() if isinstance(v, dict)})" | cut -c1-1500
