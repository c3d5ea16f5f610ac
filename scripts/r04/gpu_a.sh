#!/bin/bash
# Round-4 pass A (baseline, before the one-sided restructure): whole-round
# times of the one-sided lane (exact) next to ipc_fused_lite at 64 / 256 MiB,
# 4 processes on the card; config 4's fast-rank median; a per-rank kernel
# trace of the one-sided 256 MiB rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r04a
mkdir -p $O/base $O/trace
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=4 --master-addr 127.0.0.1 \
  --master-port 29610 bench/onesided_round.py --sizes-mb 64,256 --straggler --out-dir $O/base \
  > $O/base.log 2>&1 || { echo "base rc=$?"; tail -30 $O/base.log; exit 1; }
python - <<'PY'
import json
rows=[json.load(open(f"gpurun_out/r04a/base/rank{i}.json")) for i in range(4)]
for j,c in enumerate(rows[0]["cases"]):
    ms=max(r["cases"][j].get("ms",0) for r in rows)
    print(c["lane"], c["size_mb"], "exact", c.get("exact"), "max ms", round(ms,4), "algbw", round(c["size_mb"]*2**20/ms/1e6,1), c.get("exception",""))
print(json.dumps(rows[0].get("cfg4"))[:1500])
PY
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node=4 --master-addr 127.0.0.1 \
  --master-port 29611 --no-python rocprofv3 --kernel-trace --stats -d $O/trace -o run \
  -- python bench/onesided_round.py --sizes-mb 64,256 --lanes onesided --steps 5 --out-dir $O/trace \
  > $O/trace.log 2>&1 || { echo "trace rc=$?"; tail -30 $O/trace.log; exit 1; }
find $O/trace -name "*kernel_stats.csv" | head -1 | xargs head -12 | cut -c1-200
