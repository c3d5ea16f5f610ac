#!/bin/bash
# Round-5 pass P: push copy variants of the one-sided lane (AKKA_OS_PUSH_PL:
# 0 = 8-vector batches, 1 = software-pipelined 4-vector batches, 2 =
# pipelined 8, 3 = 4-vector batches (round-4 push)), same box A/B,
# window output, 4 and 2 ranks on the card, 64 / 256 MiB.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
O=gpurun_out/r05/p
mkdir -p $O
port=29960
for NP in 4 2; do
  for PL in 3 0 1 3 0 1; do
    port=$((port+1)); T=n${NP}_pl${PL}_$port; mkdir -p $O/$T
    AKKA_OS_PUSH_PL=$PL timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node=$NP \
      --master-addr 127.0.0.1 --master-port $port bench/onesided_round.py --sizes-mb 64,256 --lanes onesided_wo \
      --steps 20 --warmup 5 --out-dir $O/$T > $O/$T.log 2>&1 || { echo "$T rc=$?"; tail -30 $O/$T.log; exit 1; }
    python - <<PY
import json
d = json.load(open("$O/$T/rank0.json"))
print("$T", [(c["size_mb"], round(c["ms"], 4)) for c in d["cases"]] if isinstance(d, dict) and "cases" in d else str(d)[:300])
PY
  done
done
