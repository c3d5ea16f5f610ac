"""Which host reads of a lane's device memory wait for its running call?"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")
import numpy as np  # noqa: E402
import torch  # noqa: E402

from akka_allreduce_amd._native_loader import load  # noqa: E402

nat = load()
dev = torch.device("cuda", 0)
lanes = [nat.OneSidedLane(0, 12, 4, 1, r, "float32", th_reduce=0.75, th_complete=0.75, max_lag=5,
                          part_bytes=1 << 40, timeout_ms=3000) for r in range(4)]
hs = [ln.handle() for ln in lanes]
for ln in lanes:
    ln.open(hs)
for ln in lanes:
    ln.peek_flags(), ln.stats_nowait()
torch.cuda.synchronize()
w = lanes[0]
s = torch.cuda.Stream(dev)
x = torch.ones(12, device=dev)
out = torch.empty(12, device=dev)
counts = torch.empty((4, 3), dtype=torch.int32, device=dev)
torch.cuda.synchronize()
t0 = time.perf_counter()
call = w.round(s.cuda_stream, x.data_ptr(), out.data_ptr(), counts.data_ptr(), 3)
time.sleep(0.05)
for name, fn in [("peer peek_flags", lambda: lanes[1].peek_flags()),
                 ("worker peek_flags", lambda: w.peek_flags()),
                 ("peer stats_nowait", lambda: lanes[1].stats_nowait()),
                 ("worker stats_nowait", lambda: w.stats_nowait()),
                 ("worker info", lambda: w.info()),
                 ("inject", lambda: lanes[1].inject(0, 0, 0, 0, 0, 0, np.ones(1, np.float32).tobytes()))]:
    ts = time.perf_counter()
    fn()
    print(f"{name}: {1e3 * (time.perf_counter() - ts):.1f} ms (t={time.perf_counter() - t0:.3f}s)", flush=True)
s.synchronize()
print("call done at", time.perf_counter() - t0, w.status(call), flush=True)
