#!/bin/bash
# Round-3 GPU pass AI: N=1 headline pass, more workgroups (grid cap 16 -> 32
# / 64 blocks per CU), alternating with the default, one box.
set -o pipefail
mkdir -p gpurun_out/r03ai
for i in 1 2; do
  for cfg in "16 4" "32 4" "64 4" "64 2"; do
    set -- $cfg
    env AKKA_VEC_BPC=$1 AKKA_VEC_UNROLL=$2 timeout -k 10 120 python -u bench/n1_bigcopy.py 268435456 fp32 \
      | sed "s/^{/{\"bpc_set\": $1, \"unroll\": $2, /" >> gpurun_out/r03ai/sweep.jsonl || exit 1
  done
done
