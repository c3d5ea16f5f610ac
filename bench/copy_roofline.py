#!/usr/bin/env python3
"""HBM roofline for the N=1 round (a 1-source reduce = a copy): our reduce
kernel vs torch's device copy (hipMemcpy D2D) at buffer sizes below and above
the 256 MiB Infinity Cache.  Bandwidth counts read + write bytes."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from akka_allreduce_amd.ops import chunk_reduce  # noqa: E402


def t_ms(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


for mb in (64, 256, 1024, 4096):
    n = mb * (1 << 20) // 4
    x = torch.randn(n, device="cuda")
    y = torch.empty_like(x)
    row = {"MiB": mb}
    for name, fn in (("reduce_vec", lambda: chunk_reduce([x], out=y, impl="vec")),
                     ("reduce_lds", lambda: chunk_reduce([x], out=y, impl="lds")),
                     ("torch_copy", lambda: y.copy_(x))):
        ms = t_ms(fn)
        row[name + "_TBps"] = round(2 * mb * (1 << 20) / (ms * 1e-3) / 1e12, 3)
    print(json.dumps(row), flush=True)
    del x, y
