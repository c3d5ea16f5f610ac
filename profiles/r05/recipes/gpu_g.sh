#!/bin/bash
# Round-5 pass G: TCC bytes of one round (rank 0 under counter collection, 4
# processes on the card; TCC counters are device-wide, so a dispatch window
# of rank 0 also counts the other ranks' traffic): WRITE_SIZE and FETCH_SIZE
# per lane at 256 MiB -- the one-sided lane with its gather copy, with the
# window output, and the direct ipc round.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
export TMPDIR=/tmp
O=gpurun_out/r05/g
mkdir -p $O
i=0
for L in onesided onesided_wo ipc_direct; do
  for C in WRITE_SIZE FETCH_SIZE; do
    i=$((i+1)); mkdir -p $O/p_${L}_$C $O/o_${L}_$C
    PMC=$C PMC_DIR=$O/p_${L}_$C timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node=4 \
      --master-addr 127.0.0.1 --master-port $((29800+i)) --no-python bash scripts/pmc_rank0.sh \
      bench/onesided_round.py --sizes-mb 256 --lanes $L --ipc-lane ipc_fused_lite --steps 4 --warmup 1 \
      --out-dir $O/o_${L}_$C > $O/p_${L}_$C.log 2>&1 || { echo "pmc $L $C rc=$?"; grep -v "^    @" $O/p_${L}_$C.log | tail -20; exit 1; }
  done
  echo "== $L"
  python scripts/pmc_summary.py $O/p_${L}_WRITE_SIZE $O/p_${L}_FETCH_SIZE | tee $O/pmc_$L.txt
done
