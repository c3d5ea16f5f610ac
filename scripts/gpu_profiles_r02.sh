#!/bin/bash
# Round-2 profile pass: kernel traces of the N=8 shape rehearsal (p2p exact
# schedule through real RCCL on one GPU) and of the reactive 3-rank loopback.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
O=$R/gpurun_out/prof_r02
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/shape -o shape -- python3 $R/bench/host_overhead_shape.py --ns 8 --modes exact_steps --rounds 20 > $O/shape.log 2>&1 || { echo "shape rc=$?"; tail -5 $O/shape.log; exit 1; }
python3 $R/scripts/prof_summary.py $O/shape/shape_results.db 25 > $O/shape_summary.txt 2>&1 || ls -R $O/shape | head
head -30 $O/shape_summary.txt
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/react -o react -- python3 $R/bench/straggler_gpu.py --n 3 --size-mb 256 --chunk-mb 4 --th 1.0 --delay-ms 0 --rounds 10 --modes reactive > $O/react.log 2>&1 || { echo "react rc=$?"; tail -5 $O/react.log; exit 1; }
python3 $R/scripts/prof_summary.py $O/react/react_results.db 25 > $O/react_summary.txt 2>&1 || ls -R $O/react | head
head -30 $O/react_summary.txt
