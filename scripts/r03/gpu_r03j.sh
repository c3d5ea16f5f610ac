#!/bin/bash
# Round-3 GPU pass J: bench.py's cfg3 takes 28.5 ms per 1 GiB bf16 round on the
# fused lite ipc lane while the matrix (sync, chunk S/16) took 3.2 ms: isolate
# chunk size and async_op.
set -o pipefail
mkdir -p gpurun_out/r03j
timeout -k 10 900 python -u scripts/ipc_round_matrix.py --cases \
"4:536870912:bfloat16:fused:1:1024:4194304:0,4:536870912:bfloat16:fused:1:1024:4194304:1,4:536870912:bfloat16:fused:1:1024:0:1,4:67108864:float32:fused:1:1024:1048576:1" \
  > gpurun_out/r03j/matrix.jsonl 2> gpurun_out/r03j/matrix.err
