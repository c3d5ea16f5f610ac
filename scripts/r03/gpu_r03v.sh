#!/bin/bash
# Round-3 GPU pass V: the big-stream (1 GiB bf16, N=1 config 3) policy at
# 1-3 blocks per CU x 2/4/8 vectors per lane; bench.py N=1 line after the
# change (headline + cfg3).
set -o pipefail
mkdir -p gpurun_out/r03v
for u in 2 4 8; do
  for b in 1 2 3; do
    env AKKA_VEC_UNROLL=$u AKKA_VEC_BPC=$b timeout -k 10 120 python -u bench/n1_bigcopy.py 1073741824 bf16 \
      | sed "s/^{/{\"unroll\": $u, /" >> gpurun_out/r03v/bigcopy.jsonl || exit 1
  done
done
timeout -k 10 300 python bench.py > gpurun_out/r03v/bench_n1.json 2> gpurun_out/r03v/bench_n1.err
