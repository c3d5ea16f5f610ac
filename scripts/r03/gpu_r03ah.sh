#!/bin/bash
# Round-3 GPU pass AH: the N=1 headline's pass (256 MiB fp32, one source,
# cache-resident input, nontemporal stores) per blocks/CU x vectors per lane,
# alternating with the default, one box.
set -o pipefail
mkdir -p gpurun_out/r03ah
for cfg in "16 4" "8 4" "4 4" "8 8" "4 8" "2 8" "16 2" "32 4"; do
  set -- $cfg
  env AKKA_VEC_BPC=$1 AKKA_VEC_UNROLL=$2 timeout -k 10 120 python -u bench/n1_bigcopy.py 268435456 fp32 \
    | sed "s/^{/{\"bpc_set\": $1, \"unroll\": $2, /" >> gpurun_out/r03ah/sweep.jsonl || exit 1
done
timeout -k 10 120 python -u bench/n1_bigcopy.py 268435456 fp32 | sed 's/^{/{"bpc_set": "default", /' >> gpurun_out/r03ah/sweep.jsonl
