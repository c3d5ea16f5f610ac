#!/bin/bash
# Round-2 GPU pass: tests, smoke, bench, counter inventory, small-chunk reduce sweep.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
STEPS="${STEPS:-pytest smoke bench counters sweep}"
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
step pytest 900 bash -c "python -u -m pytest -q --timeout 120 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1; rc=\$?; tail -4 $O/pytest_gpu.log; exit \$rc"
step smoke 200 bash -c "python __graft_entry__.py smoke > $O/smoke.log 2>&1; rc=\$?; tail -1 $O/smoke.log; exit \$rc"
step bench 300 bash -c "python bench.py > $O/bench1.json 2> $O/bench1.err; rc=\$?; cat $O/bench1.json; exit \$rc"
step counters 120 bash -c "rocprofv3 --list-avail > $O/counters_avail.txt 2>&1; grep -iE 'RDREQ|WRREQ|EA0|FETCH|TCC_HIT|TCC_MISS' $O/counters_avail.txt | head -80"
step sweep 300 bash -c "for b in 2 4 8 16; do AKKA_VEC_BPC=\$b python bench/reduce_kernel_bw.py --sizes-mb 4,8 --nsrc 8 --dtypes float32 --impls vec,vec_nts,lds --iters 50 2>/dev/null | sed \"s/^/bpc=\$b /\"; done > $O/sweep_small.txt; cat $O/sweep_small.txt"
exit 0
