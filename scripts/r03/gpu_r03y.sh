#!/bin/bash
# Round-3 GPU pass Y: column sum with padded LDS staging: tests, timing,
# LDS bank-conflict counter.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r03y
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_step_gpu.py \
  > $O/pytest.log 2>&1 &&
timeout -k 10 200 python -u bench/colsum_bw.py > $O/colsum.jsonl 2> $O/colsum.err &&
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS \
  --output-format csv -d $O/p1 -o run -- python3 $R/bench/cfg5_step.py --dtype bf16 --graph --steps 10 --warmup 3 \
  > $O/p1.log 2>&1) &&
python3 $R/scripts/pmc_summary.py $O/p1 > $O/summary.txt 2>&1
