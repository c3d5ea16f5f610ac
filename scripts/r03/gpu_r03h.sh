#!/bin/bash
# Round-3 GPU pass H: whole exact ipc rounds, 4 processes sharing the card,
# size x dtype x phase-2 mode x lite (cfg3's 1 GiB bf16 ran 6x slower per byte
# than the 256 MiB fp32 headline in pass G).
set -o pipefail
mkdir -p gpurun_out/r03h
timeout -k 10 900 python -u scripts/ipc_round_matrix.py --cases \
"4:67108864:float32:fused:1:1024,4:134217728:bfloat16:fused:1:1024,4:268435456:float32:fused:1:1024,4:536870912:bfloat16:fused:1:1024,4:536870912:bfloat16:pull:1:1024,4:536870912:bfloat16:pull:0:256,4:268435456:float32:pull:1:1024" \
  > gpurun_out/r03h/matrix.jsonl 2> gpurun_out/r03h/matrix.err
[ $? -eq 0 ] || exit 1
R=$(pwd)
timeout -k 10 200 python -u bench/cfg5_step.py --dtype fp32 > gpurun_out/r03h/cfg5_fp32.json 2>&1 &&
timeout -k 10 200 python -u bench/cfg5_step.py --dtype bf16 > gpurun_out/r03h/cfg5_bf16.json 2>&1 &&
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d $R/gpurun_out/r03h/cfg5_trace -o run -- python3 $R/bench/cfg5_step.py --dtype bf16 --steps 30 \
  > $R/gpurun_out/r03h/cfg5_trace.log 2>&1)
