#!/usr/bin/env python3
"""Microbenchmark of the gfx950 chunk-reduce kernel variants (vec vs LDS-DMA).

Reports achieved HBM bandwidth = (nsrc reads + 1 write) * bytes / time, per
variant / source count / chunk size, as JSON lines (one per configuration).
Also times the torch reference (torch.stack(...).sum) for context.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from akka_allreduce_amd.ops import chunk_reduce


def time_fn(fn, iters: int) -> float:
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--sizes-mb", default="4,32,256")
    p.add_argument("--impls", default="vec,lds", help="comma list: auto,vec,lds,vec_nts,vec_ntl,vec_both")
    p.add_argument("--nsrc", default="1,2,4,8")
    p.add_argument("--dtypes", default="float32,bfloat16")
    p.add_argument("--iters", type=int, default=20)
    p.add_argument("--torch-ref", action="store_true")
    a = p.parse_args()
    dev = torch.device("cuda")
    for dt_name in a.dtypes.split(","):
        dt = getattr(torch, dt_name)
        es = torch.finfo(dt).bits // 8
        for mb in [float(x) for x in a.sizes_mb.split(",")]:
            n = int(mb * (1 << 20)) // es
            for k in [int(x) for x in a.nsrc.split(",")]:
                srcs = [torch.randn(n, device=dev).to(dt) for _ in range(k)]
                out = torch.empty_like(srcs[0])
                bytes_moved = (k + 1) * n * es
                row = {"dtype": dt_name, "chunk_mb": mb, "nsrc": k}
                for impl in a.impls.split(","):
                    t = time_fn(lambda: chunk_reduce(srcs, out=out, impl=impl), a.iters)
                    row[f"{impl}_us"] = round(t * 1e6, 2)
                    row[f"{impl}_GBps"] = round(bytes_moved / t / 1e9, 1)
                if a.torch_ref:
                    t = time_fn(lambda: torch.stack(srcs).float().sum(0).to(dt), max(3, a.iters // 4))
                    row["torch_GBps"] = round(bytes_moved / t / 1e9, 1)
                print(json.dumps(row), flush=True)
                del srcs, out


if __name__ == "__main__":
    main()
