#!/bin/bash
# Round 6: kernel + HIP API trace of 64 Ki-element exact rounds, 2 ranks on
# the card, one job per lane (engine-path ipc round vs its direct launch vs
# the one-sided lane): what the GPU does between two rounds of each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06/${1:-small_trace}
mkdir -p $O
port=29631
for L in ${LANES:-ipc_fused_lite ipc_fused_lite_direct onesided}; do
  port=$((port+1))
  rm -rf $O/trace_$L
  timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 \
    --master-port $port --no-python rocprofv3 --kernel-trace --hip-trace --output-format csv -d $O/trace_$L \
    -o run_%pid% -- python bench/small_rounds.py --mode nk --sizes 65536 --lanes $L --calls 100 \
    > $O/trace_$L.log 2>&1 || { echo "trace $L rc=$?"; tail -30 $O/trace_$L.log; exit 1; }
  echo "== $L"
  grep '"lane"' $O/trace_$L.log | head -2
  python scripts/engine_path_trace.py $O/trace_$L --split-ms 2 --min-rounds 50 --json $O/trace_$L.json \
    | tee $O/trace_$L.txt | head -12
  python scripts/r06/api_per_round.py $O/trace_$L | tee $O/api_$L.txt
done
