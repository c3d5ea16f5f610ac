#!/bin/bash
# Round 6 (final kernel): the chaos check at 15 ranks (16 processes with the launcher
# are over the box limit; the runtime-N round kernel): thresholds 1/2 and exact
# (window output), 200 rounds each, every output chunk checked.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06/${1:-chaos15}
mkdir -p $O
port=30600
for V in "n15_th05:0.5:2:" "n15_exact_wo:1.0:1:--window-output"; do
  IFS=: read -r tag th lag extra <<< "$V"
  port=$((port+1)); mkdir -p $O/$tag
  timeout -k 10 280 python -m torch.distributed.run --nnodes=1 --nproc-per-node=15 --master-addr 127.0.0.1 \
    --master-port $port tests/onesided_ranks.py --out-dir $O/$tag --device cuda --mode chaos --th $th --max-lag $lag \
    --rounds 200 --jitter-ms 1 --size $((1 << 22)) --chunk $((1 << 18)) --timeout-s 20 $extra > $O/$tag.log 2>&1 \
    || { echo "$tag rc=$?"; tail -20 $O/$tag.log; exit 1; }
  python - "$O/$tag" 15 "$tag" <<'PY'
import json, sys
d, n, tag = sys.argv[1], int(sys.argv[2]), sys.argv[3]
rows = [json.load(open(f"{d}/rank{i}.json")) for i in range(n)]
bad = sum(r["chaos"]["bad_chunks"] for r in rows)
tmo = sum(r["chaos"]["stats"].get("timeouts", 0) for r in rows)
last = min(r["chaos"]["rounds"][-1] for r in rows)
calls = sum(len(r["chaos"]["rounds"]) for r in rows)
conf = sum(r["chaos"]["stats"]["scatter_conflict"] + r["chaos"]["stats"]["gather_conflict"] for r in rows)
print(f"{tag}: calls {calls} last_round {last} bad_chunks {bad} timeouts {tmo} conflicts {conf}")
PY
done
