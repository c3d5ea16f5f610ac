#!/bin/bash
# Round-4 pass S: bench.py N=1 with config 1 only (README demo: CPU workers
# over TCP, and GPU workers on the one-sided lane under the actor API).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r04s
mkdir -p $O
timeout -k 10 400 python bench.py --extras on --extras-only cfg1 --steps 5 --warmup 2 > $O/bench_cfg1.json \
  2> $O/bench_cfg1.err || { echo "bench rc=$?"; tail -30 $O/bench_cfg1.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_cfg1.json')); print(json.dumps(d['extra_configs'], indent=1)[:2500])"
