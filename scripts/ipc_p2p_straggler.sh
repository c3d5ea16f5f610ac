#!/bin/bash
# Reactive transport over the mailbox p2p, 4 processes on one card, rank 3 a
# straggler: per-round times of every rank (tests/p2p_ranks.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/p2p_straggler
for cfg in "0 1 8" "300 1 8" "300 64 8" "300 64 6"; do
  set -- $cfg
  d=gpurun_out/p2p_straggler/delay$1_mb$2_q$3
  mkdir -p $d
  GPU_MAX_HW_QUEUES=$3 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node=4 \
    --master-addr 127.0.0.1 --master-port $((29700 + $1 % 7 + $2 % 5 + $3)) tests/p2p_ranks.py --out-dir $d \
    --transport reactive --th 0.75 --size $(( $2 * 262144 )) --chunk 1048576 --rounds 8 --straggler-ms $1 \
    > $d/log.txt 2>&1 || { echo "cfg $cfg failed"; tail -5 $d/log.txt; exit 1; }
  python - "$d" "$cfg" <<'PY'
import json, sys
d, cfg = sys.argv[1], sys.argv[2]
rows = [json.load(open(f"{d}/rank{i}.json")) for i in range(4)]
print(f"delay_ms,MiB,queues={cfg}: " + " | ".join(f"r{r['rank']} {r['ms_per_round']}" for r in rows))
PY
done
