#!/bin/bash
# Round 6 final kernel: the N=4 one-sided exact round (window output) next to
# the direct ipc round, 256 MiB, 4 processes on the card (as os_shares.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06/${1:-os_n4_final}
mkdir -p $O
port=29881
for L in ipc_direct onesided_wo onesided; do
  port=$((port+1))
  mkdir -p $O/$L
  timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node=4 --master-addr 127.0.0.1 \
    --master-port $port bench/onesided_round.py --sizes-mb 64,256 --lanes $L --ipc-lane ipc_fused_lite \
    --steps 20 --warmup 5 --out-dir $O/$L > $O/$L.log 2>&1 || { echo "$L rc=$?"; tail -30 $O/$L.log; exit 1; }
done
python - $O <<'PY' | tee $O/summary.txt
import json, glob, sys
rows = {}
for f in glob.glob(sys.argv[1] + "/*/rank*.json"):
    for c in json.load(open(f))["cases"]:
        rows.setdefault((c["lane"], c["size_mb"]), []).append(c.get("ms"))
for (lane, mb), v in sorted(rows.items(), key=lambda kv: (kv[0][1], kv[0][0])):
    print("%-26s %6g MiB %8.4f ms" % (lane, mb, max(v)))
PY
