#!/usr/bin/env python3
"""HIP-graph replay of a threshold-allreduce round (N=1 on one MI355X, or any N
under torchrun): capture ``ar(x, out=buf)`` once with ``torch.cuda.graph``
(relaxed capture -- the engine queries events while it schedules), then
``replay()`` re-runs the round's GPU work without the host engine.  Valid for
exact thresholds with fixed buffers, where every round does the same work.
Prints eager vs replay time per round for small (launch-bound) buffers."""
from __future__ import annotations

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from akka_allreduce_amd.parallel import ThresholdAllreduce  # noqa: E402


def main():
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
    torch.cuda.set_device(dev)
    for kib in (64, 1024, 16384):
        S = kib * 1024 // 4
        ar = ThresholdAllreduce(S, max_chunk_size=min(S, 1 << 20), device=dev)
        x = torch.randn(S, device=dev)
        buf = torch.empty(S, device=dev)
        for _ in range(5):
            ar(x, out=buf)
        torch.cuda.synchronize()
        iters = 200
        t0 = time.perf_counter()
        for _ in range(iters):
            ar(x, out=buf)
        torch.cuda.synchronize()
        eager = (time.perf_counter() - t0) / iters
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s, capture_error_mode="relaxed"):
                out = ar(x, out=buf)
        torch.cuda.synchronize()
        x.copy_(torch.arange(S, device=dev, dtype=torch.float32))
        g.replay()
        torch.cuda.synchronize()
        ok = bool(torch.equal(out.data, x)) and bool((out.count == ar.world_size).all())
        t0 = time.perf_counter()
        for _ in range(iters):
            g.replay()
        torch.cuda.synchronize()
        replay = (time.perf_counter() - t0) / iters
        # a loop of K rounds captured in one graph: one graph launch per K rounds
        K = 16
        gk = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            with torch.cuda.graph(gk, stream=s, capture_error_mode="relaxed"):
                for _ in range(K):
                    outk = ar(x, out=buf)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(iters // K):
            gk.replay()
        torch.cuda.synchronize()
        loop = (time.perf_counter() - t0) / ((iters // K) * K)
        ok &= bool(torch.equal(outk.data, x))
        print(json.dumps({"KiB": kib, "eager_us": round(eager * 1e6, 2), "replay_us": round(replay * 1e6, 2),
                          f"replay_{K}_rounds_per_graph_us": round(loop * 1e6, 2),
                          "speedup_loop": round(eager / loop, 2), "exact_after_replay": ok}), flush=True)


if __name__ == "__main__":
    main()
