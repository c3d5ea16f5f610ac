#!/usr/bin/env python3
"""BASELINE config 4: threshold allreduce (thReduce 0.75, thComplete 0.75,
maxLag 1) with one induced straggler.

--mode cluster (default when no GPU / WORLD_SIZE=1): master + N message-driven
   workers (TCP actor nodes, CPU data plane); the last worker's data source
   sleeps --delay-ms per round.  Reports rounds/s with and without the
   straggler and the mean contributor count: rounds complete without waiting
   for the slow worker (thAllreduce pacing + thresholds + maxLag catch-up).
--mode spmd (under torch.distributed.run on GPUs): rank N-1 sleeps before each
   call.  --transport stream (scheduled RCCL steps, a rendezvous: the delay is
   paid by every rank) or --transport reactive (per-peer streams + pair
   communicators: the fast ranks' own time per round is reported separately).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

if "reactive" in sys.argv:
    os.environ["GPU_MAX_HW_QUEUES"] = "32"  # per-peer streams (read at HIP init)

import torch  # noqa: E402


def run_cluster(a) -> dict:
    from akka_allreduce_amd.config import DataConfig, ThresholdConfig, WorkerConfig
    from akka_allreduce_amd.data import AllReduceInput
    from akka_allreduce_amd.parallel.cluster import start_master, start_worker
    from akka_allreduce_amd.utils.metrics import MetricsSink

    res = {}
    for straggle in (False, True):
        m = start_master(ThresholdConfig(a.th_allreduce, a.th_reduce, a.th_complete),
                         DataConfig(a.size, a.chunk, a.rounds), WorkerConfig(a.workers, a.max_lag), port=0,
                         transport="tcp", unreachable_after_s=60)
        sinks, ws = [], []
        for i in range(a.workers):
            slow = straggle and i == a.workers - 1
            data = torch.arange(a.size, dtype=torch.float32)

            def src(req, slow=slow, data=data):
                if slow:
                    time.sleep(a.delay_ms / 1e3)
                return AllReduceInput(data)

            sink = MetricsSink(with_counts=True)
            sinks.append(sink)
            ws.append(start_worker(m.address, a.size, data_source=src, data_sink=sink))
        t0 = time.time()
        ok = m.wait(300)
        dt = time.time() - t0
        live = sinks[:-1] if straggle else sinks
        mean_count = sum(r["count_mean"] for s in live for r in s.rows) / max(1, sum(len(s.rows) for s in live))
        res["straggler" if straggle else "baseline"] = {
            "finished": ok, "rounds_per_s": round(a.rounds / dt, 2), "mean_contributors": round(mean_count, 3),
            "straggler_rounds_delivered": len(sinks[-1].rows)}
        m.stop()
        for w in ws:
            w.stop()
        time.sleep(0.2)
    return res


def run_spmd(a) -> dict:
    import torch.distributed as dist

    from akka_allreduce_amd.parallel import ThresholdAllreduce

    rank, world = int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1 and not dist.is_initialized():
        dist.init_process_group("gloo", rank=rank, world_size=world)
    S = int(a.size_mb * (1 << 20)) // 4
    ar = ThresholdAllreduce(S, max_chunk_size=(4 << 20) // 4, th_reduce=a.th_reduce, th_complete=a.th_complete,
                            max_lag=a.max_lag, device=dev, transport=a.transport)
    x = torch.randn(S, device=dev)
    res = {}
    for straggle in (False, True):
        for _ in range(3):
            ar(x)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(a.rounds):
            if straggle and rank == world - 1:
                time.sleep(a.delay_ms / 1e3)
            out = ar(x)
        torch.cuda.synchronize()
        own = time.perf_counter() - t0  # this rank's own time for the rounds
        ar.drain()
        if world > 1:
            dist.barrier()
        dt = time.perf_counter() - t0
        owns = [own]
        if world > 1:
            owns = [None] * world
            dist.all_gather_object(owns, own)
        fast = max(owns[:-1]) if world > 1 else own
        res["straggler" if straggle else "baseline"] = {
            "rounds_per_s": round(a.rounds / dt, 2), "algbw_GBps": round(S * 4 * a.rounds / dt / 1e9, 2),
            "fast_ranks_ms_per_round": round(fast / a.rounds * 1e3, 3),
            "mean_contributors": float(out.count.float().mean())}
    res["transport"] = a.transport
    return res


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--mode", choices=["auto", "cluster", "spmd"], default="auto")
    p.add_argument("--workers", type=int, default=4)
    p.add_argument("--size", type=int, default=1 << 16)
    p.add_argument("--size-mb", type=float, default=64)
    p.add_argument("--chunk", type=int, default=4096)
    p.add_argument("--rounds", type=int, default=100)
    p.add_argument("--delay-ms", type=float, default=20.0)
    p.add_argument("--th-allreduce", type=float, default=0.75)
    p.add_argument("--th-reduce", type=float, default=0.75)
    p.add_argument("--th-complete", type=float, default=0.75)
    p.add_argument("--max-lag", type=int, default=1)
    p.add_argument("--transport", choices=["stream", "reactive"], default="stream", help="spmd mode data path")
    a = p.parse_args()
    mode = a.mode
    if mode == "auto":
        mode = "spmd" if int(os.environ.get("WORLD_SIZE", "1")) > 1 and torch.cuda.is_available() else "cluster"
    res = run_cluster(a) if mode == "cluster" else run_spmd(a)
    if int(os.environ.get("RANK", "0")) == 0:
        print(json.dumps({"config": "threshold allreduce with one straggler", "mode": mode,
                          "thresholds": [a.th_allreduce, a.th_reduce, a.th_complete], "maxLag": a.max_lag,
                          "delay_ms": a.delay_ms, **res}), flush=True)


if __name__ == "__main__":
    main()
