#!/bin/bash
# Round-6 chaos campaign (copy-role verdict flag fixed) of the one-sided lane on the GPU
# (tests/onesided_ranks.py --mode chaos): every rank waits U(0, 1 ms) before
# each call, 1000 rounds per run, several (N, thresholds, maxLag) shapes, both
# hand-off modes, two jitter seeds; exact shapes also with window output.
# Every output chunk of every call is checked (one contributor set matching
# its count); prints one summary line per run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06/${1:-chaos}
mkdir -p $O
port=30000
run() {  # tag n th lag extra...
  local tag=$1 n=$2 th=$3 lag=$4; shift 4
  port=$((port+1)); mkdir -p $O/$tag
  timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node=$n --master-addr 127.0.0.1 \
    --master-port $port tests/onesided_ranks.py --out-dir $O/$tag --device cuda --mode chaos --th $th --max-lag $lag \
    --rounds 1000 --jitter-ms ${JITTER:-1} --size $((1 << 22)) --chunk $((1 << 18)) --timeout-s 10 "$@" > $O/$tag.log 2>&1 \
    || { echo "$tag rc=$?"; tail -20 $O/$tag.log; return 1; }
  python - "$O/$tag" "$n" "$tag" <<'PY'
import json, sys
d, n, tag = sys.argv[1], int(sys.argv[2]), sys.argv[3]
rows = [json.load(open(f"{d}/rank{i}.json")) for i in range(n)]
bad = sum(r["chaos"]["bad_chunks"] for r in rows)
tmo = sum(r["chaos"]["stats"].get("timeouts", 0) for r in rows)
err = sum(r["error"] for r in rows)
last = min(r["chaos"]["rounds"][-1] for r in rows)
part = sum(r["chaos"]["calls_with_partial_chunks"] for r in rows)
calls = sum(len(r["chaos"]["rounds"]) for r in rows)
st = rows[0]["chaos"]["stats"]
print(f"{tag}: calls {calls} last_round {last} bad_chunks {bad} timeouts {tmo} errors {err} partial_calls {part} "
      f"conflicts {st.get('scatter_conflict', st.get('scatterConflict', '?'))}")
if bad or tmo or err or last < 999:
    sys.exit(1)
PY
}
# the shape whose run caught the copy-role race (8 ranks, bf16, th 0.5, lite), 2 ms jitter
JITTER=2 run n8_th05_l2_lite_j2_s3 8 0.5 2 --handoff lite --seed 3 --dtype bfloat16 || exit 1
JITTER=2 run n8_th05_l2_lite_j2_s4 8 0.5 2 --handoff lite --seed 4 --dtype bfloat16 || exit 1
for seed in 1 2; do
  for h in lite fenced; do
    run n8_th05_l2_${h}_s$seed 8 0.5 2 --handoff $h --seed $seed --dtype bfloat16 && \
    run n4_th075_l1_${h}_s$seed 4 0.75 1 --handoff $h --seed $seed && \
    run n5_th06_l3_${h}_s$seed 5 0.6 3 --handoff $h --seed $seed && \
    run n8_exact_wo_${h}_s$seed 8 1.0 1 --handoff $h --seed $seed --window-output || exit 1
  done
done
