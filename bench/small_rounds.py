#!/usr/bin/env python3
"""Small-round cost: where the host time of one exact round goes.

``--mode n1`` (one process): per-call host microseconds of
``ThresholdAllreduce.__call__`` at N=1, and of each piece of that call on its
own (stream lookup, counts allocation, the native ``fast_round``, the output
object, a bare kernel launch of the same copy), at 64 Ki and 64 Mi elements.

``--mode nk`` (torch.distributed.run, ranks sharing the box's GPU or one GPU
each): per-call host and wall microseconds of the engine-path ipc round
(synchronous calls), the direct launch of the same kernel and the one-sided
lane at 64 Ki elements, plus the same breakdown of the engine call.

Rank 0 prints one JSON line per case; ``--out`` also writes them to a file.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def _per_call(fn, calls: int) -> float:
    t0 = time.perf_counter()
    for _ in range(calls):
        fn()
    return (time.perf_counter() - t0) / calls * 1e6


def _sync_loop(fn, calls: int, dev) -> tuple[float, float]:
    """(host us per call, wall us per call) over `calls` back-to-back calls."""
    torch.cuda.synchronize(dev)
    host = 0.0
    t0 = time.perf_counter()
    for _ in range(calls):
        a = time.perf_counter()
        fn()
        host += time.perf_counter() - a
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    return host / calls * 1e6, wall / calls * 1e6


def _latency(fn, calls: int, dev) -> float:
    """us per call when every call is waited for (round trip)."""
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(calls):
        fn()
        torch.cuda.synchronize(dev)
    return (time.perf_counter() - t0) / calls * 1e6


def pieces(ar, x, buf, calls: int) -> dict:
    """The pieces of one engine call, each timed on its own."""
    from akka_allreduce_amd._native_loader import load
    from akka_allreduce_amd.data import AllReduceOutput

    w = ar.worker
    dev = x.device
    g = w.geometry
    core = w._core
    n = load()
    res = {}
    res["current_stream_us"] = _per_call(lambda: torch.cuda.current_stream(dev), calls)
    res["cuda_stream_attr_us"] = _per_call(lambda: torch.cuda.current_stream(dev).cuda_stream, calls)
    res["torch_empty_counts_us"] = _per_call(lambda: torch.empty(g.workerNum * g.kmax, dtype=torch.int32, device=dev),
                                             calls)
    counts = torch.empty(g.workerNum * g.kmax, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    xp, bp, cp = x.data_ptr(), buf.data_ptr(), counts.data_ptr()

    def native():
        r = w._next_round
        w._next_round += 1
        core.fast_round(r, xp, bp, cp, s, True)

    res["native_fast_round_us"] = _sync_loop(native, calls, dev)[0]
    res["output_object_us"] = _per_call(
        lambda: AllReduceOutput(buf, iteration=0, counts_per_chunk=counts.view(g.workerNum, g.kmax), geometry=g,
                                expander=None, event=None), calls)
    res["fast_ok_us"] = _per_call(lambda: w._fast_ok(x), calls)
    res["data_ptr_x3_us"] = _per_call(lambda: (x.data_ptr(), buf.data_ptr(), counts.data_ptr()), calls)
    if g.workerNum == 1:
        res["bare_reduce_launch_us"] = _sync_loop(lambda: n.reduce(bp, [xp], x.numel(), "float32", s), calls, dev)[0]
    res["torch_copy_launch_us"] = _sync_loop(lambda: buf.copy_(x), calls, dev)[0]
    res["event_record_us"] = _per_call(lambda: torch.cuda.Event().record(), calls)
    return res


def mode_n1(args) -> list:
    from akka_allreduce_amd.parallel import ThresholdAllreduce

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    rows = []
    for S in [int(v) for v in args.sizes.split(",")]:
        ar = ThresholdAllreduce(S, max_chunk_size=1 << 20, device=dev, rank=0, world_size=1)
        x = torch.randn(S, device=dev)
        buf = torch.empty_like(x)
        for _ in range(20):
            ar(x, out=buf)
        host, wall = _sync_loop(lambda: ar(x, out=buf), args.calls, dev)
        lat = _latency(lambda: ar(x, out=buf), max(20, args.calls // 4), dev)
        ok = bool(torch.equal(ar(x, out=buf).data, x))
        row = {"mode": "n1", "elements": S, "host_us_per_call": round(host, 2), "wall_us_per_call": round(wall, 2),
               "latency_us": round(lat, 2), "exact": ok}
        row.update({k: round(v, 2) for k, v in pieces(ar, x, buf, args.calls).items()})
        rows.append(row)
    return rows


def mode_n1seg(args) -> list:
    """The N=1 call path of ThresholdAllreduce.__call__ replayed inline with a
    clock between its segments, like bench.py's timed loop (``--calls``
    back-to-back calls after 5 warm-ups): where the host microseconds go."""
    from akka_allreduce_amd.data import AllReduceOutput
    from akka_allreduce_amd.parallel import ThresholdAllreduce
    from akka_allreduce_amd.worker import _raw_stream

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    rows = []
    pc = time.perf_counter_ns
    for S in [int(v) for v in args.sizes.split(",")]:
        ar = ThresholdAllreduce(S, max_chunk_size=1 << 20, device=dev, rank=0, world_size=1)
        w = ar.worker
        g = w.geometry
        x = torch.randn(S, device=dev)
        buf = torch.empty_like(x)
        for _ in range(5):
            ar(x, out=buf)
        torch.cuda.synchronize(dev)
        seg = {k: 0 for k in ("checks", "counts", "stream", "native", "output", "total")}
        for _ in range(args.calls):
            t0 = pc()
            ok = (x.numel() == ar.data_size and w is not None and ar.pacer is None and ar._direct is None
                  and not ar._lane_os and not ar._ipc_direct and not ar.fault_delay_s and w._fast_ok(x)
                  and w._buffer_ok(buf))
            t1 = pc()
            counts = w._counts_by_out.get(buf.data_ptr())
            if counts is None:
                counts = w._counts_for(buf)
            r = w._next_round
            w._next_round += 1
            t2 = pc()
            sptr = _raw_stream(w._dev_index)
            t3 = pc()
            done = w._core.fast_round(r, x.data_ptr(), buf.data_ptr(), counts.data_ptr(), sptr, True)
            t4 = pc()
            o = AllReduceOutput._make(buf, done[0], counts, g, w._expand_counts, None)
            t5 = pc()
            assert ok and o is not None
            for k, a, b in (("checks", t0, t1), ("counts", t1, t2), ("stream", t2, t3), ("native", t3, t4),
                            ("output", t4, t5), ("total", t0, t5)):
                seg[k] += b - a
        torch.cuda.synchronize(dev)
        row = {"mode": "n1seg", "elements": S, **{k + "_us": round(v / args.calls / 1e3, 2) for k, v in seg.items()}}
        host, _ = _sync_loop(lambda: ar(x, out=buf), args.calls, dev)
        row["full_call_us"] = round(host, 2)
        rows.append(row)
    return rows


def mode_nk(args) -> list:
    import torch.distributed as dist

    from akka_allreduce_amd.parallel import ThresholdAllreduce

    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    ndev = torch.cuda.device_count()
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", rank)) % ndev)
    torch.cuda.set_device(dev)
    rows = []
    S = int(args.sizes.split(",")[0])
    x = torch.randn(S, device=dev)
    buf = torch.empty_like(x)
    if args.user_stream:  # every call on a stream of the caller's making (not the default stream)
        torch.cuda.set_stream(torch.cuda.Stream(dev))
    for spec in args.lanes.split(","):
        # "<lane>[+devrounds][+finish]": measurement variants of the ipc lanes --
        # engine rounds reading their id from device memory (the direct
        # launch's bump kernel), direct rounds writing the counts table in
        # their last workgroup (the engine round's finish_counts)
        name, *opts = spec.split("+")
        if name == "onesided":
            ar = ThresholdAllreduce(S, max_chunk_size=1 << 14, device=dev, transport="onesided")
        else:
            ar = ThresholdAllreduce(S, max_chunk_size=1 << 14, device=dev, data_plane="ipc")
            ar.use_lane(name)
            if "devrounds" in opts:
                ar.worker._core.ipc_device_rounds(True)
            if "finish" in opts:
                ar._ipc_finish = True
        for _ in range(20):
            ar(x, out=buf)
        torch.cuda.synchronize(dev)
        dist.barrier()
        host, wall = _sync_loop(lambda: ar(x, out=buf), args.calls, dev)
        dist.barrier()
        lat = _latency(lambda: ar(x, out=buf), max(20, args.calls // 4), dev)
        o = ar(torch.full((S,), float(rank + 1), device=dev), out=buf)
        torch.cuda.synchronize(dev)
        ok = bool(torch.all(o.data == world * (world + 1) / 2).item())
        row = {"mode": f"n{world}", "lane": spec, "elements": S, "host_us_per_call": round(host, 2),
               "wall_us_per_call": round(wall, 2), "latency_us": round(lat, 2), "exact": ok,
               "gpus": ndev}
        ipc = ar.state().get("link", {}).get("ipc") if name != "onesided" else None
        if ipc:
            row["windows_id"] = hex(ipc["windows_id"])
        if name != "onesided" and not name.endswith("_direct") and not opts:
            dist.barrier()
            row.update({k: round(v, 2) for k, v in pieces(ar, x, buf, args.calls).items()
                        if k in ("native_fast_round_us", "torch_empty_counts_us", "current_stream_us")})
        torch.cuda.synchronize(dev)
        dist.barrier()
        if rank == 0:
            rows.append(row)
        if args.free:
            del o  # (the output holds the engine: free its windows before the next lane's)
        del ar
    dist.destroy_process_group()
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=("n1", "n1seg", "nk"), default="n1")
    ap.add_argument("--sizes", default="65536,67108864")
    ap.add_argument("--calls", type=int, default=400)
    ap.add_argument("--lanes", default="ipc_fused_lite,ipc_fused_lite_direct,onesided")
    ap.add_argument("--out", default="")
    ap.add_argument("--free", action="store_true", help="nk: free each lane before creating the next")
    ap.add_argument("--user-stream", action="store_true", help="nk: run the calls on a user-created stream")
    args = ap.parse_args()
    rows = {"n1": mode_n1, "n1seg": mode_n1seg, "nk": mode_nk}[args.mode](args)
    for r in rows:
        print(json.dumps(r), flush=True)
    if args.out and rows:
        os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
        with open(args.out, "a") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
