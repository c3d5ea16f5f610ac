#!/bin/bash
# Round-3 GPU pass AG: same-box A/B of the one-source big-stream policy:
# old (4 blocks/CU x 2 vectors) vs new default (2 x 4), alternating.
set -o pipefail
mkdir -p gpurun_out/r03ag
for i in 1 2 3; do
  env AKKA_VEC_BPC=4 AKKA_VEC_UNROLL=2 timeout -k 10 120 python -u bench/n1_bigcopy.py 1073741824 bf16 \
    | sed 's/^{/{"policy": "old_b4_u2", /' >> gpurun_out/r03ag/ab.jsonl || exit 1
  timeout -k 10 120 python -u bench/n1_bigcopy.py 1073741824 bf16 \
    | sed 's/^{/{"policy": "new_default", /' >> gpurun_out/r03ag/ab.jsonl || exit 1
done
