#!/bin/bash
# One GPU-box pass: gpu tests, smoke, 1-GPU bench, kernel microbench, rocprof.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
O=$R/gpurun_out
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
echo "== env"; (rocm-smi --showproductname 2>/dev/null | head -20; python -c "import torch;print(torch.__version__, torch.cuda.get_device_name(0))") > $O/env.txt 2>&1
echo "== pytest -m gpu" && timeout -k 10 600 python -m pytest tests -m gpu -q --maxfail=10 > $O/pytest_gpu.log 2>&1; rc=$?; tail -5 $O/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
echo "== smoke" && timeout -k 10 300 python __graft_entry__.py smoke > $O/smoke.log 2>&1 && tail -2 $O/smoke.log \
&& echo "== bench" && timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench1.json 2> $O/bench1.err && cat $O/bench1.json \
&& echo "== reduce microbench" && timeout -k 10 300 python bench/reduce_kernel_bw.py --torch-ref > $O/reduce_bw.jsonl 2>&1 && cat $O/reduce_bw.jsonl \
&& echo "== rocprof" && cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o bench -- python $R/bench.py --steps 10 --warmup 3 > $O/prof.log 2>&1; echo "rocprof rc=$?"
exit $rc
