#!/bin/bash
# Round-4 pass C: config 5's eager step, round-1 tree (ab/r01, its own
# extension) vs HEAD, alternating on one box; then a HIP API trace of each
# (runtime trace only, no counters) to count host API calls per step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r04c
mkdir -p $O
for i in 1 2 3; do
  for t in ab/r01 .; do
    timeout -k 10 180 python bench/cfg5_ab.py --root $t --steps 50 >> $O/ab.jsonl 2> $O/ab_err.log \
      || { echo "ab $t rc=$?"; tail -20 $O/ab_err.log; exit 1; }
  done
done
cat $O/ab.jsonl
for t in r01 head; do
  root=ab/r01; [ $t = head ] && root=.
  timeout -k 10 240 rocprofv3 --hip-trace --kernel-trace --stats --output-format csv -d $O/trace_$t -o run \
    -- python bench/cfg5_ab.py --root $root --steps 20 --warmup 5 > $O/trace_$t.log 2>&1 \
    || { echo "trace $t rc=$?"; tail -20 $O/trace_$t.log; exit 1; }
done
find $O -name "*hip_api_stats.csv" | while read f; do echo "== $f"; head -25 "$f" | cut -c1-160; done
