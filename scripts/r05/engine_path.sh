#!/bin/bash
# Engine path vs direct launch of the exact ipc round:
# kernel trace of bench/onesided_round.py with 4 processes on the card,
# ipc_fused_lite through the engine and the same lane launched directly,
# 64 and 256 MiB; per-round timeline by scripts/engine_path_trace.py.
# Usage: scripts/r05/engine_path.sh <out-tag> [ipc lane]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05/${1:-engine_path}
LANE=${2:-ipc_fused_lite}
mkdir -p $O/trace $O/ot
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node=4 --master-addr 127.0.0.1 \
  --master-port 29701 --no-python rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run_%pid% \
  -- python bench/onesided_round.py --sizes-mb 64,256 --lanes ipc,ipc_direct,onesided --ipc-lane $LANE \
  --steps 12 --warmup 3 --out-dir $O/ot > $O/trace.log 2>&1 || { echo "trace rc=$?"; tail -30 $O/trace.log; exit 1; }
python scripts/engine_path_trace.py $O/trace --json $O/engine_path.json | tee $O/engine_path.txt
python - <<PY
import json, glob
for f in sorted(glob.glob("$O/ot/rank*.json")):
    d = json.load(open(f))
    print(d["rank"], [(c["lane"], c["size_mb"], c.get("ms"), c.get("exact"), c.get("exception")) for c in d["cases"]])
PY
