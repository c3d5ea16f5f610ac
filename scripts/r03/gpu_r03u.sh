#!/bin/bash
# Round-3 GPU pass U: config 3's N=1 round (1 GiB bf16 one-source pass) per
# load/store policy and blocks per CU, vs torch copy_; smoke(); bench
# contract (link probe now one launch per iteration on one stream).
set -o pipefail
mkdir -p gpurun_out/r03u
for b in auto 2 4 8 16; do
  if [ $b = auto ]; then E=""; else E="AKKA_VEC_BPC=$b"; fi
  env $E timeout -k 10 120 python -u bench/n1_bigcopy.py 1073741824 bf16 >> gpurun_out/r03u/bigcopy.jsonl 2>/dev/null || exit 1
done
timeout -k 10 120 python -u bench/n1_bigcopy.py 268435456 fp32 >> gpurun_out/r03u/bigcopy.jsonl 2>/dev/null &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03u/smoke.log 2>&1 &&
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_bench_contract_gpu.py \
  > gpurun_out/r03u/pytest_contract.log 2>&1
