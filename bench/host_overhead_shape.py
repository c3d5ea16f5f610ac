#!/usr/bin/env python3
"""Host cost per round of the N-rank scheduled transport, rehearsed on ONE
MI355X (RcclShapeP2P: a 1-rank RCCL communicator posing as rank 0 of N, every
op sent to itself -- the bytes are meaningless, the engine / link / RCCL
enqueue path and the group shapes are the real ones).

For N = 2, 4, 8 at the headline geometry (256 MiB fp32, 4 MiB chunks, lag 2:
kmax + 2 steps, 4(N-1) ops per step) it times
  * exact_steps    -- exact thresholds: the per-geometry op template
                      (stream_link.cpp exact_steps), no engine callbacks,
  * message_flow   -- thReduce just below 1: the engine's per-chunk message
                      flow drives the same schedule (plus counts exchange),
and prints host microseconds spent inside allreduce() per round (the number
that decides whether N=8 rounds are host-bound) and GPU ms per round (self
copies here, not xGMI).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from akka_allreduce_amd import AllreduceWorker, InitWorkers  # noqa: E402
from akka_allreduce_amd.parallel.collective import _RemoteRank  # noqa: E402


def run(n: int, mode: str, size_mb: float, chunk_mb: float, rounds: int, graphs: bool) -> dict:
    dev = torch.device("cuda", 0)
    S = int(size_mb * (1 << 20)) // 4
    C = int(chunk_mb * (1 << 20)) // 4
    w = AllreduceWorker(None, None, device=dev, transport="stream", transport_spec=("rccl_shape", 0, n),
                        broadcast_lag=2, strict=True, name=f"shape{n}")
    th = 1.0 if mode == "exact_steps" else 1.0 - 0.5 / n
    peers = {i: (w if i == 0 else _RemoteRank(i)) for i in range(n)}
    w.tell(InitWorkers(peers, n, None, 0, th, 1.0, 2, S, C))
    w.set_lane("p2p")
    if graphs:
        w.set_graphs(True)
    x = torch.randn(S, device=dev)
    out = torch.empty_like(x)
    for _ in range(5):
        o = w.allreduce(x, async_op=True, out=out)
    o.wait()
    torch.cuda.synchronize()
    host = 0.0
    t0 = time.perf_counter()
    for _ in range(rounds):
        th0 = time.perf_counter()
        o = w.allreduce(x, async_op=True, out=out)
        host += time.perf_counter() - th0
    o.wait()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    st = w.state()
    link = st["link"]
    res = {"n_shape": n, "mode": mode, "graphs": graphs, "buffer_MiB": size_mb, "chunk_MiB": chunk_mb,
           "groups_per_round": round(link["groups"] / max(1, link["rounds"]), 2),
           "ops_per_round": round(link["ops"] / max(1, link["rounds"]), 1),
           "host_us_per_round": round(host / rounds * 1e6, 1),
           "gpu_ms_per_round": round(wall / rounds * 1e3, 3),
           "exact_step_rounds": link.get("exact_step_rounds"), "graph_replays": link.get("graph_replays")}
    w.close()
    return res


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--size-mb", type=float, default=256.0)
    p.add_argument("--chunk-mb", type=float, default=4.0)
    p.add_argument("--rounds", type=int, default=30)
    p.add_argument("--ns", default="2,4,8")
    p.add_argument("--modes", default="message_flow,exact_steps,exact_steps+graphs")
    a = p.parse_args()
    for n in [int(v) for v in a.ns.split(",")]:
        for m in a.modes.split(","):
            graphs = m.endswith("+graphs")
            print(json.dumps(run(n, m.replace("+graphs", ""), a.size_mb, a.chunk_mb, a.rounds, graphs)), flush=True)


if __name__ == "__main__":
    main()
