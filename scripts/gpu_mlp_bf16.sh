set -o pipefail
O=gpurun_out/${OUTDIR:-s4b}; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_collective_gpu.py tests/test_mlp_cpu.py > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python examples/mlp_sgd.py > $O/mlp_fp32.json 2>&1 && tail -1 $O/mlp_fp32.json &&
timeout -k 10 200 python examples/mlp_sgd.py --compute-dtype bfloat16 > $O/mlp_bf16.json 2>&1 && tail -1 $O/mlp_bf16.json &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err && cat $O/bench.json &&
cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o mlp -- python $GRAFT_REPO_ROOT/examples/mlp_sgd.py --compute-dtype bfloat16 --steps 20 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 && python $GRAFT_REPO_ROOT/scripts/prof_summary.py $GRAFT_REPO_ROOT/$O/prof/mlp_results.db 25 > $GRAFT_REPO_ROOT/$O/prof_mlp_bf16.txt 2>&1; head -14 $GRAFT_REPO_ROOT/$O/prof_mlp_bf16.txt
