#!/bin/bash
# Round-4 pass H: raw TCC byte counters of the one-sided round per buffer size
# (rank 0 under counter collection, 4 processes on the card; one counter and
# one size per pass), then the whole GPU suite, smoke(), bench.py N=1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r04h
mkdir -p $O
i=0
for S in 64 256; do
  for C in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1)); mkdir -p $O/s${S}_$C $O/o$i
    PMC=$C PMC_DIR=$O/s${S}_$C timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node=4 \
      --master-addr 127.0.0.1 --master-port $((29680+i)) --no-python bash scripts/r04/pmc_rank0.sh \
      bench/onesided_round.py --sizes-mb $S --lanes onesided,ipc --steps 6 --warmup 2 --out-dir $O/o$i \
      > $O/p$i.log 2>&1 || { echo "pmc $S $C rc=$?"; grep -v "^    @" $O/p$i.log | tail -20; exit 1; }
  done
  echo "== $S MiB"; python scripts/pmc_summary.py $O/s${S}_FETCH_SIZE $O/s${S}_WRITE_SIZE | grep -E "os_|ipc_fused" | tee $O/pmc_${S}.txt
done
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench_n1.json 2> $O/bench_n1.err || { echo "bench rc=$?"; tail -20 $O/bench_n1.err; exit 1; }
cut -c1-400 $O/bench_n1.json
