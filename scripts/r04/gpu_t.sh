#!/bin/bash
# Round-4 pass T: per-role timeline of the one-sided round (4 ranks on the
# card, exact, 64 / 256 MiB), from the kernel's per-workgroup clock stamps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r04t
mkdir -p $O/tl
timeout -k 10 200 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=4 --master-addr 127.0.0.1 \
  --master-port 29790 bench/onesided_timeline.py --out-dir $O/tl > $O/tl.log 2>&1 \
  || { echo "tl rc=$?"; grep -v Warning $O/tl.log | tail -30; exit 1; }
grep '^{' $O/tl.log | grep '"rank": 0' 
