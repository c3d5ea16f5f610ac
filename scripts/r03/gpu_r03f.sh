#!/bin/bash
# Round-3 GPU pass F: raw TCC/EA counters of the reduce role (fenced vs lite,
# N=8, 32 MiB, 512 KiB portions, 1024 threads), a kernel-trace summary of the
# same, and a 1-GPU bench.py run.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out/r03f
PMC_OUT=r03f/pmc PMC_BENCH_ARGS="--n 2,8 --block-mb 32 --threads 1024 --portion-kb 512 --modes sys,lite" \
  timeout -k 10 400 bash scripts/pmc_ipc_reduce.sh > gpurun_out/r03f/pmc.log 2>&1 &&
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r03f/ktrace -o run \
  -- python3 $R/bench/ipc_reduce_role.py --n 8 --block-mb 32 --threads 1024 --portion-kb 512 --modes sys,lite \
  > $R/gpurun_out/r03f/ktrace.log 2>&1) &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r03f/bench_n1.json 2> gpurun_out/r03f/bench_n1.err
