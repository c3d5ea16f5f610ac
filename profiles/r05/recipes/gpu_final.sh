#!/bin/bash
# Round-5 final pass: the whole GPU suite + smoke() (what the driver runs at
# round end), then bench.py N=1 (the driver's BENCH run) and a rocprofv3
# kernel-trace --stats of it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
O=gpurun_out/r05/final
mkdir -p $O
timeout -k 10 1000 python -u -m pytest -v --timeout 240 --timeout-method thread -m gpu tests/ > $O/pytest.txt 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/pytest.txt | tail -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 300 python bench.py > $O/bench_n1.json 2> $O/bench_n1.err || { tail -20 $O/bench_n1.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_n1.json')); print(d['value'], d['ms_per_step'], d.get('extra_configs', {}).keys())"
mkdir -p $O/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o n1 -- python bench.py --steps 20 --warmup 5 --extras off > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
echo prof ok
