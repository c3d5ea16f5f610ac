#!/bin/bash
# Round-3 GPU pass G: new GPU tests (N=8 ipc-lite and onesided kernels, DDP
# hook on the onesided lane), then bench.py's N-rank flow with 4 processes
# sharing the card on the ipc data plane (lane selection incl. lite lanes,
# link probe, cfg4 on the onesided lane).
set -o pipefail
mkdir -p gpurun_out/r03g
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  "tests/test_ipc_gpu.py::test_ipc_lane_lite_handoffs" "tests/test_onesided_gpu.py::test_onesided_gpu_exact_rounds" \
  "tests/test_dp_ipc_gpu.py::test_torch_ddp_hook_onesided_multiprocess" > gpurun_out/r03g/pytest.log 2>&1 &&
AKKA_SHARE_GPU=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 4 --data-plane ipc --steps 10 --warmup 3 \
  > gpurun_out/r03g/bench_shared_n4_ipc.json 2> gpurun_out/r03g/bench_shared_n4_ipc.err
