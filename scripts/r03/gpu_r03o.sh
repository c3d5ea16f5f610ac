#!/bin/bash
# Round-3 GPU pass O: why a second (idle) engine in each of 4 processes
# sharing the card slows the 1 GiB bf16 ipc round 2x (8x with
# GPU_MAX_HW_QUEUES=2, pass N): engine created without rounds, engine deleted
# before the timed one, more hardware queues, comm stream at normal priority.
set -o pipefail
mkdir -p gpurun_out/r03o
C=4:536870912:bfloat16:pull:0:256:4194304:1
timeout -k 10 600 python -u scripts/ipc_round_matrix.py --cases \
"$C:67108864:0:0,$C:67108864:5:1,$C:67108864:5:0" \
  > gpurun_out/r03o/matrix_a.jsonl 2> gpurun_out/r03o/matrix_a.err &&
timeout -k 10 300 python -u scripts/ipc_round_matrix.py --env "GPU_MAX_HW_QUEUES=8" --cases "$C:67108864:5:0" \
  > gpurun_out/r03o/matrix_hwq8.jsonl 2> gpurun_out/r03o/matrix_hwq8.err &&
timeout -k 10 400 python -u scripts/ipc_round_matrix.py --env "AKKA_COMM_PRIORITY=normal" \
  --cases "$C:67108864:5:0,$C:0" > gpurun_out/r03o/matrix_prio.jsonl 2> gpurun_out/r03o/matrix_prio.err
