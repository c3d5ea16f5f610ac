#!/bin/bash
# Round-5 pass K: the one-sided lane's bounded footprint (cu_keep on a GPU of
# its own, AKKA_OS_DEDICATED=1 standing in on this 1-GPU box): torch DDP
# steps on the one-sided transport (2 ranks on the card, bench/ddp_overlap.py)
# -- sync without a mask, sync with the small grid, async and sync rounds
# with the bounded footprint -- and a kernel trace of the sync one-sided DDP
# step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
O=gpurun_out/r05/k
mkdir -p $O
i=0
one() {  # tag, extra env (k=v, may be empty), args...
  i=$((i+1)); tag=$1; ev=$2; shift 2
  env AKKA_SHARE_GPU=1 GPU_MAX_HW_QUEUES=8 $ev timeout -k 10 150 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node=2 --master-addr 127.0.0.1 --master-port $((29870+i)) bench/ddp_overlap.py "$@" > $O/$tag.log 2>&1 \
    || { echo "$tag rc=$?"; tail -20 $O/$tag.log; return 1; }
  echo "$tag $(grep ms_per_step $O/$tag.log)"
}
# (bounded runs: AKKA_OS_ROLE_WGS=48 keeps BOTH ranks' grids resident on the
# kept CUs of this one card -- sized as on a GPU of its own, one rank's grid
# alone would fill them and hold the slots the other rank's pushers need)
B="AKKA_OS_DEDICATED=1 AKKA_OS_ROLE_WGS=48"
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_dp_ipc_gpu.py tests/test_ddp_hook_gpu.py > $O/pytest.txt 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/pytest.txt | tail -8
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|assert" $O/pytest.txt | head -60; exit $rc; }
one os_sync_nomask "" --transport onesided --cu-keep 0 --modes sync && \
one os_sync_wgs48 "AKKA_OS_ROLE_WGS=48" --transport onesided --cu-keep 0 --modes sync && \
one os_async_bounded4 "$B" --transport onesided --cu-keep 4 --modes async && \
one os_sync_bounded4 "$B" --transport onesided --cu-keep 4 --modes sync && \
one os_async_bounded6 "$B" --transport onesided --cu-keep 6 --modes async || exit 1
mkdir -p $O/trace_os_sync
AKKA_SHARE_GPU=1 GPU_MAX_HW_QUEUES=8 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 \
  --master-addr 127.0.0.1 --master-port 29899 --no-python rocprofv3 --kernel-trace --stats --output-format csv \
  -d $O/trace_os_sync -o run_%pid% -- python bench/ddp_overlap.py --transport onesided --cu-keep 0 --modes sync \
  --steps 10 --warmup 3 > $O/trace_os_sync.log 2>&1 || { echo "trace rc=$?"; tail -20 $O/trace_os_sync.log; exit 1; }
grep ms_per_step $O/trace_os_sync.log
