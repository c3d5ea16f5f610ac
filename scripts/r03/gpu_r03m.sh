#!/bin/bash
# Round-3 GPU pass M (fresh container): N=1 headline on this tree, then the
# cfg3 bisect of pass L (1 GiB bf16 ipc round with / without another engine
# in the process first).
set -o pipefail
mkdir -p gpurun_out/r03m
timeout -k 10 300 python bench.py > gpurun_out/r03m/bench_n1.json 2> gpurun_out/r03m/bench_n1.err &&
timeout -k 10 600 python -u scripts/ipc_round_matrix.py --cases \
"4:536870912:bfloat16:pull:0:256:4194304:1:67108864,4:536870912:bfloat16:pull:0:256:4194304:1:0" \
  > gpurun_out/r03m/matrix.jsonl 2> gpurun_out/r03m/matrix.err
