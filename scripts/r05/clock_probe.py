"""How long does a one-sided wait of timeout T really take on this GPU?
A worker lane (spec harness, same process) waits for copies that never come;
its call must end after ~T with reason "timeout".  Prints the measured time
per T and the lane's clock rate (hipDeviceAttributeWallClockRate, kHz)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests"))
import torch  # noqa: E402

from akka_allreduce_amd._native_loader import load  # noqa: E402

nat = load()
dev = torch.device("cuda", 0)
for T_ms in (500, 2000):
    lanes = [nat.OneSidedLane(0, 8, 2, 2, r, "float32", th_reduce=1.0, th_complete=1.0, max_lag=1,
                              part_bytes=1 << 40, timeout_ms=T_ms) for r in range(2)]
    hs = [ln.handle() for ln in lanes]
    for ln in lanes:
        ln.open(hs)
    w = lanes[0]
    s = torch.cuda.Stream(dev)
    x = torch.ones(8, device=dev)
    out = torch.empty(8, device=dev)
    counts = torch.empty((2, 4), dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    call = w.round(s.cuda_stream, x.data_ptr(), out.data_ptr(), counts.data_ptr(), 4)
    s.synchronize()
    dt = time.perf_counter() - t0
    print(f"timeout {T_ms} ms -> call took {dt * 1e3:.1f} ms, status {w.status(call)}, clock_khz {w.info()['clock_khz']}",
          flush=True)
