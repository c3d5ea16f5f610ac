#!/bin/bash
# Round-4 pass AA: 256- vs 1024-thread workgroups of the one-sided round on
# the shared card (N=2 and N=4, exact, 64 / 256 MiB).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r04aa
mkdir -p $O
i=0
for N in 2 4; do
  for T in 256 1024; do
    i=$((i+1)); mkdir -p $O/v$i
    AKKA_OS_THREADS=$T timeout -k 10 200 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=$N \
      --master-addr 127.0.0.1 --master-port $((29830+i)) bench/onesided_round.py --sizes-mb 64,256 --lanes onesided \
      --out-dir $O/v$i > $O/v$i.log 2>&1 || { echo "v$i rc=$?"; tail -20 $O/v$i.log; exit 1; }
    echo "== N=$N threads $T"; python scripts/r04/summarize_round.py $O/v$i $N | tee $O/v$i.jsonl | cut -c1-200
  done
done
