#!/bin/bash
# Engine path vs direct launch of the exact ipc round,
# 4 processes on the card, 64 and 256 MiB fp32, lane $2 (ipc_fused_lite):
#   * timing: bench/onesided_round.py, one job per lane variant (engine async,
#     engine sync, direct, onesided), no profiler;
#   * trace: the same jobs under rocprofv3 --kernel-trace, per-round
#     timeline by scripts/engine_path_trace.py.
# Usage: profiles/r05/recipes/engine_path.sh <out-tag> [ipc lane] [sizes]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
O=gpurun_out/r05/${1:-engine_path}
LANE=${2:-ipc_fused_lite}
SIZES=${3:-64,256}
mkdir -p $O
port=29701
for L in ${LANES:-ipc ipc_sync ipc_direct onesided}; do
  mkdir -p $O/time_$L $O/trace_$L $O/ot_$L
  port=$((port+1))
  timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node=4 --master-addr 127.0.0.1 \
    --master-port $port bench/onesided_round.py --sizes-mb $SIZES --lanes $L --ipc-lane $LANE --steps 20 --warmup 5 \
    --out-dir $O/time_$L > $O/time_$L.log 2>&1 || { echo "time $L rc=$?"; tail -30 $O/time_$L.log; exit 1; }
  port=$((port+1))
  timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node=4 --master-addr 127.0.0.1 \
    --master-port $port --no-python rocprofv3 --kernel-trace --output-format csv -d $O/trace_$L -o run_%pid% \
    -- python bench/onesided_round.py --sizes-mb $SIZES --lanes $L --ipc-lane $LANE --steps 12 --warmup 3 \
    --out-dir $O/ot_$L > $O/trace_$L.log 2>&1 || { echo "trace $L rc=$?"; tail -30 $O/trace_$L.log; exit 1; }
  echo "== $L"
  python scripts/engine_path_trace.py $O/trace_$L --json $O/trace_$L.json | tee $O/trace_$L.txt | grep "run 0\|run 1" | head -4
done
python - <<PY | tee $O/summary.txt
import json, glob
rows = {}
for L in "${LANES:-ipc ipc_sync ipc_direct onesided}".split():
    for f in sorted(glob.glob("$O/time_%s/rank*.json" % L)):
        d = json.load(open(f))
        for c in d["cases"]:
            rows.setdefault((c["lane"], c["size_mb"]), []).append(c.get("ms"))
print("%-28s %8s %12s" % ("lane", "MiB", "ms (max rank)"))
for (lane, mb), v in sorted(rows.items(), key=lambda kv: (kv[0][1], kv[0][0])):
    print("%-28s %8g %12.4f" % (lane, mb, max(x for x in v if x is not None)))
PY
