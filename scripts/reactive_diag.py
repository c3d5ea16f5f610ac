"""Diagnose the reactive loopback on one GPU: N ranks, small rounds, with a
watchdog that dumps every thread's stack and hard-exits instead of hanging.

usage: reactive_diag.py N S [dtype] [clusters]
"""
import faulthandler
import os
import sys
import time

os.environ["GPU_MAX_HW_QUEUES"] = "32"  # the box exports 4
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from akka_allreduce_amd.parallel.loopback import ReactiveLoopbackCluster  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 3
S = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
dt = {"f32": torch.float32, "bf16": torch.bfloat16}[sys.argv[3] if len(sys.argv) > 3 else "f32"]
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 1
print("GPU_MAX_HW_QUEUES", os.environ.get("GPU_MAX_HW_QUEUES"), "n", n, "S", S, dt, "clusters", reps, flush=True)
faulthandler.enable(all_threads=True)
faulthandler.dump_traceback_later(40, exit=True)
for rep in range(reps):
    with ReactiveLoopbackCluster(n, S, 4096, max_lag=1, dtype=dt) as cl:
        rounds = [[torch.full((S,), float(1 << i), device="cuda", dtype=dt) for i in range(n)] for _ in range(2)]
        t0 = time.time()
        outs = cl.run_rounds(rounds, timeout=15)
        torch.cuda.synchronize()
        print(rep, "ok", round(time.time() - t0, 4), [o.data[0].item() for o in outs[0]], flush=True)
faulthandler.cancel_dump_traceback_later()
print("done", flush=True)
os._exit(0)
