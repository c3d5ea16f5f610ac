#!/bin/bash
# Round 6: engine-path async rounds vs the direct launch:
# 4 processes on the card, 64 / 256 MiB fp32, ipc_fused_lite, one job per
# lane variant (engine async, engine sync, direct), timing only.
# Usage: scripts/r06/engine_async.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06/${1:-engine_async}
mkdir -p $O
port=29801
for L in ${LANES:-ipc ipc_sync ipc_direct}; do
  mkdir -p $O/time_$L
  port=$((port+1))
  timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node=${NPROC:-4} --master-addr 127.0.0.1 \
    --master-port $port bench/onesided_round.py --sizes-mb ${SIZES:-64,256} --lanes $L --ipc-lane ipc_fused_lite \
    --steps 20 --warmup 5 --out-dir $O/time_$L > $O/time_$L.log 2>&1 || { echo "time $L rc=$?"; tail -30 $O/time_$L.log; exit 1; }
done
python - <<PY | tee $O/summary.txt
import json, glob
rows = {}
for L in "${LANES:-ipc ipc_sync ipc_direct}".split():
    for f in sorted(glob.glob("$O/time_%s/rank*.json" % L)):
        d = json.load(open(f))
        for c in d["cases"]:
            rows.setdefault((c["lane"], c["size_mb"]), []).append(c.get("ms"))
print("%-28s %8s %12s" % ("lane", "MiB", "ms (max rank)"))
for (lane, mb), v in sorted(rows.items(), key=lambda kv: (kv[0][1], kv[0][0])):
    print("%-28s %8g %12.4f" % (lane, mb, max(x for x in v if x is not None)))
PY
