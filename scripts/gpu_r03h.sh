#!/bin/bash
# Round-3 GPU pass H: whole exact ipc rounds, 4 processes sharing the card,
# size x dtype x phase-2 mode x lite (cfg3's 1 GiB bf16 ran 6x slower per byte
# than the 256 MiB fp32 headline in pass G).
set -o pipefail
mkdir -p gpurun_out/r03h
timeout -k 10 900 python -u scripts/ipc_round_matrix.py --cases \
"4:67108864:float32:fused:1:1024,4:134217728:bfloat16:fused:1:1024,4:268435456:float32:fused:1:1024,4:536870912:bfloat16:fused:1:1024,4:536870912:bfloat16:pull:1:1024,4:536870912:bfloat16:pull:0:256,4:268435456:float32:pull:1:1024" \
  > gpurun_out/r03h/matrix.jsonl 2> gpurun_out/r03h/matrix.err
