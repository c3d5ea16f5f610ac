set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dp_rep
for mem in fine fine fine coarse; do
  AKKA_IPC_MEM=$mem timeout -k 10 200 python -m pytest -x -q --timeout 180 --timeout-method thread "tests/test_dp_ipc_gpu.py::test_dp_sgd_multiprocess_ipc" > gpurun_out/dp_rep/$mem.log 2>&1
  echo "mem=$mem rc=$? $(tail -1 gpurun_out/dp_rep/$mem.log)"
  grep -E "Greatest|Mismatched" gpurun_out/dp_rep/$mem.log | head -3 || true
done
exit 0
