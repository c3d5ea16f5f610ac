#!/bin/bash
# Round-5 pass M: the DDP hook's in-place mean (into the bucket): DDP steps
# with gradient_as_bucket_view on / off, 2 ranks on the card, the fast lanes
# (bench/ddp_overlap.py), then the DDP GPU tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
O=gpurun_out/r05/m
mkdir -p $O
i=0
one() {  # tag, args...
  i=$((i+1)); tag=$1; shift
  AKKA_SHARE_GPU=1 GPU_MAX_HW_QUEUES=8 timeout -k 10 150 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node=2 --master-addr 127.0.0.1 --master-port $((29910+i)) bench/ddp_overlap.py "$@" > $O/$tag.log 2>&1 \
    || { echo "$tag rc=$?"; tail -20 $O/$tag.log; return 1; }
  echo "$tag $(grep ms_per_step $O/$tag.log)"
}
for bv in 1 0; do
  one direct_bv$bv --transport stream --data-plane ipc --lane ipc_fused_lite_direct --modes sync --bucket-view $bv && \
  one os_bv$bv --transport onesided --cu-keep 0 --modes sync --bucket-view $bv && \
  one engine_bv$bv --transport stream --data-plane ipc --lane ipc_fused_lite --modes sync --bucket-view $bv || exit 1
done
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_dp_ipc_gpu.py tests/test_ddp_hook_gpu.py > $O/pytest.txt 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/pytest.txt | tail -8
exit $rc
