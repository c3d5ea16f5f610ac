#!/bin/bash
# Round-3 GPU pass N: config-5 step kernels (bf16 weight shadow from the fused
# update, gfx950 bias-gradient column sum) -- tests, A/B timing, kernel stats;
# then the cfg3 bisect: is the 2x slowdown with a second engine in each of 4
# processes sharing the card a hardware-queue count effect (GPU_MAX_HW_QUEUES)?
set -o pipefail
mkdir -p gpurun_out/r03n
R=$(pwd)
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fused_step_gpu.py \
  tests/test_collective_gpu.py tests/test_kernels_gpu.py > gpurun_out/r03n/pytest.log 2>&1 &&
timeout -k 10 200 python -u bench/cfg5_step.py --dtype bf16 --no-shadow > gpurun_out/r03n/cfg5.jsonl 2>&1 &&
timeout -k 10 200 python -u bench/cfg5_step.py --dtype bf16 >> gpurun_out/r03n/cfg5.jsonl 2>&1 &&
timeout -k 10 200 python -u bench/cfg5_step.py --dtype fp32 >> gpurun_out/r03n/cfg5.jsonl 2>&1 &&
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d $R/gpurun_out/r03n/cfg5_trace -o run -- python3 $R/bench/cfg5_step.py --dtype bf16 --steps 30 \
  > $R/gpurun_out/r03n/cfg5_trace.log 2>&1) &&
GPU_MAX_HW_QUEUES=2 timeout -k 10 400 python -u scripts/ipc_round_matrix.py --cases \
"4:536870912:bfloat16:pull:0:256:4194304:1:67108864,4:536870912:bfloat16:pull:0:256:4194304:1:0" \
  > gpurun_out/r03n/matrix_hwq2.jsonl 2> gpurun_out/r03n/matrix_hwq2.err
