#!/bin/bash
# Round 6: per-role timeline of a small one-sided exact round (64 Ki fp32,
# 2 ranks on the card): where its ~37 us go (bench/onesided_timeline.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06/${1:-os_small_tl}
port=29861
for PB in 0 262144; do  # auto parts vs one 256 KiB part per chunk
  port=$((port+1))
  mkdir -p $O/tl_pb$PB
  timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 \
    --master-port $port bench/onesided_timeline.py --sizes-mb 0.25 --chunk-mb 4 --calls 40 --part-bytes $PB \
    --out-dir $O/tl_pb$PB > $O/tl_pb$PB.log 2>&1 || { echo "tl rc=$?"; tail -30 $O/tl_pb$PB.log; exit 1; }
  python - $O/tl_pb$PB <<'PY'
import json, glob, statistics, sys
for f in sorted(glob.glob(sys.argv[1] + "/rank*.json")):
    r = json.load(open(f))[0]
    k = r["kernel_us_per_call"]
    b = r["fastest_call"]
    print(sys.argv[1].split("/")[-1], "rank", r["rank"], "wgs", r["role_wgs"], "median kernel us", statistics.median(k),
          "fastest", b["kernel"], {n: b[n]["last_done"] for n in ("push", "decide", "reduce", "complete", "copy")})
PY
done
