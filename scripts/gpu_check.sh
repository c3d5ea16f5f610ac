#!/bin/bash
# One GPU-box pass: gpu tests, smoke, 1-GPU bench, kernel microbench, rocprof.
# Every GPU step has its own time limit.  A step that fails normally (test
# failure, rc 1/2) does not stop the pass; a timeout, abort or crash
# (124/134/137/139) ends it immediately -- nothing more runs on the GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
O=$R/gpurun_out
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
STEPS="${STEPS:-env pytest smoke bench micro hostovh bf16 mlp rcclp2p prof}"

step() {  # step <name> <timeout-s> <cmd...>
  local name=$1 t=$2; shift 2
  case " $STEPS " in *" $name "*) ;; *) return 0 ;; esac
  echo "== $name"
  timeout -k 10 "$t" "$@"
  local rc=$?
  echo "== $name rc=$rc"
  case $rc in 124|134|137|139) echo "FATAL step $name rc=$rc: stopping"; exit $rc ;; esac
  return 0
}

step env 120 bash -c "python -c 'import torch;print(torch.__version__, torch.cuda.get_device_name(0))' > $O/env.txt 2>&1"
step reactive 400 bash -c "python -m pytest tests/test_reactive_gpu.py -q -x > $O/pytest_reactive.log 2>&1; rc=\$?; tail -15 $O/pytest_reactive.log; exit \$rc"
step pytest 900 bash -c "python -m pytest tests -m gpu -q --maxfail=20 > $O/pytest_gpu.log 2>&1; rc=\$?; tail -4 $O/pytest_gpu.log; exit \$rc"
step smoke 300 bash -c "python __graft_entry__.py smoke > $O/smoke.log 2>&1; tail -2 $O/smoke.log"
step bench 300 bash -c "python bench.py --steps 20 --warmup 5 > $O/bench1.json 2> $O/bench1.err; cat $O/bench1.json; tail -3 $O/bench1.err"
step micro 400 bash -c "python bench/reduce_kernel_bw.py --torch-ref > $O/reduce_bw.jsonl 2>&1; cat $O/reduce_bw.jsonl"
step hostovh 200 bash -c "python bench.py --steps 200 --warmup 20 --size-mb 0.0625 --chunk-mb 0.015625 --no-check > $O/bench_small.json 2>&1; cat $O/bench_small.json"
step bf16 300 bash -c "python bench.py --dtype bfloat16 --size-mb 1024 --chunk-mb 8 --steps 10 --warmup 3 > $O/bench_bf16_1g.json 2>&1; tail -1 $O/bench_bf16_1g.json"
step mlp 300 bash -c "python examples/mlp_sgd.py > $O/mlp.json 2>&1; tail -1 $O/mlp.json"
step rcclp2p 200 bash -c "python bench/rccl_p2p_overhead.py > $O/rccl_p2p.jsonl 2>&1; tail -4 $O/rccl_p2p.jsonl"
step straggler 300 bash -c "python bench/straggler_gpu.py > $O/straggler_gpu.jsonl 2>&1; rc=\$?; tail -3 $O/straggler_gpu.jsonl; exit \$rc"
step n1exp 200 bash -c "python bench/n1_experiments.py > $O/n1exp.json 2>&1; tail -2 $O/n1exp.json"
step prof 400 bash -c "cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $O/prof -o bench -- python $R/bench.py --steps 10 --warmup 3 > $O/prof.log 2>&1; tail -3 $O/prof.log; python $R/scripts/prof_summary.py $O/prof/bench_results.db 40 > $O/prof_summary.txt 2>&1; head -12 $O/prof_summary.txt"
exit 0
