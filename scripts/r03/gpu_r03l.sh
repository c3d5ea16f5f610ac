#!/bin/bash
# Round-3 GPU pass L: does a second engine in the process (bench.py's headline
# before cfg3) slow the 1 GiB bf16 ipc round down?
set -o pipefail
mkdir -p gpurun_out/r03l
timeout -k 10 600 python -u scripts/ipc_round_matrix.py --cases \
"4:536870912:bfloat16:pull:0:256:4194304:1:67108864,4:536870912:bfloat16:pull:0:256:4194304:1:0" \
  > gpurun_out/r03l/matrix.jsonl 2> gpurun_out/r03l/matrix.err
