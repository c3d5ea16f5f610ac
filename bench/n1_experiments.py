#!/usr/bin/env python3
"""Isolate the N=1 round cost: raw kernel (1 vs rotating output buffers) vs the
full engine path (async / sync, output lifetime)."""
from __future__ import annotations

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from akka_allreduce_amd.ops import chunk_reduce  # noqa: E402
from akka_allreduce_amd.parallel import ThresholdAllreduce  # noqa: E402


def timed(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e6


def main():
    dev = torch.device("cuda", 0)
    S = (256 << 20) // 4
    x = torch.randn(S, device=dev)
    res = {}
    out1 = torch.empty_like(x)
    res["kernel_single_out_us"] = timed(lambda: chunk_reduce([x], out=out1, impl="vec"))
    outs = [torch.empty_like(x) for _ in range(5)]
    k = [0]

    def rot():
        chunk_reduce([x], out=outs[k[0] % 5], impl="vec")
        k[0] += 1

    res["kernel_rotating5_us"] = timed(rot)
    res["torch_copy_us"] = timed(lambda: out1.copy_(x))

    def fresh():
        o = torch.empty_like(x)
        chunk_reduce([x], out=o, impl="vec")

    res["kernel_fresh_alloc_us"] = timed(fresh)
    ar = ThresholdAllreduce(S, max_chunk_size=1 << 20, device=dev, rank=0, world_size=1, max_lag=2)
    res["engine_sync_us"] = timed(lambda: ar(x))
    held = []

    def async_hold():
        held.append(ar(x, async_op=True))
        if len(held) > 4:
            held.pop(0).wait()

    res["engine_async_hold4_us"] = timed(async_hold)
    res["engine_async_nohold_us"] = timed(lambda: ar(x, async_op=True).wait())
    print(json.dumps({k: round(v, 1) for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
