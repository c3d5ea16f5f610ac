#!/usr/bin/env python3
"""RCCL grouped-p2p cost on ONE MI355X (1-rank communicator, self send/recv).

Measures, for the group shapes the StreamLink issues at N=2/4/8 (2 sends + 2
recvs per peer, 4 MiB each), the host time to enqueue one group and the GPU
time per group.  Self p2p is a local copy, so the GPU number is an HBM copy,
not xGMI; the HOST number is what decides whether a round at N=8 (10 groups)
is host-bound.
"""
from __future__ import annotations

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from akka_allreduce_amd._native_loader import load  # noqa: E402


def main():
    n = load()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ep = n.rccl_endpoint(n.rccl_unique_id(), 0, 1, 0)
    s = torch.cuda.Stream(dev)
    chunk = 4 << 20
    for peers in (1, 3, 7):
        nops = 2 * peers  # sends of scatter + bcast per peer (and as many recvs)
        src = [torch.randn(chunk // 4, device=dev) for _ in range(nops)]
        dst = [torch.empty_like(t) for t in src]
        ops = []
        for a, b in zip(src, dst):
            ops.append((True, 0, a.data_ptr(), chunk))
            ops.append((False, 0, b.data_ptr(), chunk))
        for _ in range(3):
            ep.group(s.cuda_stream, ops)
        torch.cuda.synchronize()
        iters = 50
        t0 = time.perf_counter()
        for _ in range(iters):
            ep.group(s.cuda_stream, ops)
        t_host = (time.perf_counter() - t0) / iters
        torch.cuda.synchronize()
        t_all = (time.perf_counter() - t0) / iters
        ok = all(torch.equal(a, b) for a, b in zip(src, dst))
        print(json.dumps({"peers_shape": peers, "ops_per_group": 2 * nops, "bytes_per_group": nops * chunk,
                          "host_us_per_group": round(t_host * 1e6, 1), "gpu_us_per_group": round(t_all * 1e6, 1),
                          "self_copy_GBps": round(nops * chunk / t_all / 1e9, 1), "correct": ok}), flush=True)


if __name__ == "__main__":
    main()
