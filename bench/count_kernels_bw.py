#!/usr/bin/env python3
"""Bandwidth of the output-side kernels against their plain-torch equivalents:

* count_expand   per-chunk counts -> int32[S]          (writes 4 B/elem)
* count_mean     sum / count  (0 where count is 0)     (reads + writes)
* axpy_mean      y += alpha * sum / count (fused SGD)  (reads 2, writes 1)

torch references: repeat_interleave for the expansion, and the same math on a
materialised per-element count tensor.  TB/s counts the bytes each kernel
must move (no count tensor for ours; the torch versions read one more).
"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from akka_allreduce_amd.data import AllReduceOutput, Geometry  # noqa: E402
from akka_allreduce_amd.ops import count_expand  # noqa: E402


def bench(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    dev = torch.device("cuda", 0)
    for mib, N, C in ((16, 8, 1 << 18), (256, 8, 1 << 20), (1024, 8, 1 << 21)):
        S = (mib << 20) // 4
        g = Geometry(S, N, C)
        d = torch.randn(S, device=dev)
        pc = torch.randint(1, N + 1, (N, g.kmax), device=dev, dtype=torch.int32)
        out = AllReduceOutput(d, counts_per_chunk=pc, geometry=g)
        y = torch.randn(S, device=dev)
        cnt = count_expand(pc, g)  # materialised once for the torch references
        b = S * 4
        rows = {
            "count_expand": (bench(lambda: count_expand(pc, g)), b),
            "count_expand_torch": (bench(lambda: pc.reshape(-1).repeat_interleave(
                torch.full((N * g.kmax,), C, device=dev))[:S]), b),
            "count_mean": (bench(lambda: AllReduceOutput(d, counts_per_chunk=pc, geometry=g).mean()), 2 * b),
            "count_mean_torch": (bench(lambda: torch.where(cnt > 0, d / cnt, torch.zeros_like(d))), 3 * b),
            "axpy_mean": (bench(lambda: out.axpy_mean_(y, -0.01)), 3 * b),
            "axpy_mean_torch": (bench(lambda: y.add_(torch.where(cnt > 0, d / cnt, torch.zeros_like(d)), alpha=-0.01)),
                                4 * b),
        }
        for k, (us, nbytes) in rows.items():
            print(json.dumps({"MiB": mib, "kernel": k, "us": round(us, 1), "TBps": round(nbytes / us / 1e6, 2)}),
                  flush=True)


if __name__ == "__main__":
    main()
