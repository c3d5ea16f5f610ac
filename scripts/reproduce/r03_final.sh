#!/bin/bash
# Round-3 final GPU pass: the whole GPU suite on the final tree (what the
# driver runs at round end), smoke(), the N=1 bench line.
set -o pipefail
mkdir -p gpurun_out/r03final
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread \
  > gpurun_out/r03final/pytest_gpu.log 2>&1 &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03final/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/r03final/bench_n1.json 2> gpurun_out/r03final/bench_n1.err
