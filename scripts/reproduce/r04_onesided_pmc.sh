#!/bin/bash
# Round-4 pass G: raw TCC byte counters of the one-sided round (rank 0 under
# counter collection, 4 processes on the card), one counter pass each; then
# bench.py's N=4 flow on the shared card (ipc data plane, lane selection with
# the onesided candidate); bench.py N=1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r04g
mkdir -p $O
mkdir -p $O/trace $O/ot
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node=4 --master-addr 127.0.0.1 \
  --master-port 29659 --no-python rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run_%pid% \
  -- python bench/onesided_round.py --sizes-mb 64,256 --lanes onesided,ipc --steps 8 --warmup 2 --out-dir $O/ot \
  > $O/trace.log 2>&1 || { echo "trace rc=$?"; tail -20 $O/trace.log; exit 1; }
python scripts/ktrace.py $O/trace 8 | tee $O/trace_summary.txt | head -40
python scripts/summarize_round.py $O/ot 4
i=0
for C in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1)); mkdir -p $O/p$i $O/o$i
  PMC=$C PMC_DIR=$O/p$i timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node=4 \
    --master-addr 127.0.0.1 --master-port $((29660+i)) --no-python bash scripts/pmc_rank0.sh \
    bench/onesided_round.py --sizes-mb 64,256 --lanes onesided,ipc --steps 3 --warmup 1 --out-dir $O/o$i \
    > $O/p$i.log 2>&1 || { echo "pmc $C rc=$?"; grep -v "^    @" $O/p$i.log | tail -20; exit 1; }
done
python scripts/pmc_summary.py $O/p1 $O/p2 | tee $O/pmc_summary.txt
AKKA_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node=4 \
  --master-addr 127.0.0.1 --master-port 29670 bench.py --gpus 4 --data-plane ipc --extras off --link-probe off \
  > $O/bench_n4_shared.json 2> $O/bench_n4_shared.err || { echo "bench n4 rc=$?"; tail -20 $O/bench_n4_shared.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_n4_shared.json')); print(d['value'], d['lane'], json.dumps(d.get('lane_select'))[:900])"
timeout -k 10 400 python bench.py > $O/bench_n1.json 2> $O/bench_n1.err || { echo "bench n1 rc=$?"; tail -20 $O/bench_n1.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_n1.json')); print(d['value'], d['ms_per_step'], json.dumps(d.get('extra_configs'))[:1500])"
