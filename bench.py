#!/usr/bin/env python3
"""Headline benchmark: allreduce algbw (GB/s) on a 256 MB fp32 buffer, 1/2/4/8 MI355X.

Metric and config come from BASELINE.json.  One rank per GPU; for N>1 the
driver launches this file under ``torch.distributed.run`` (RANK/LOCAL_RANK/
WORLD_SIZE/MASTER_* in the env).  Each timed step is one full threshold-
allreduce round through the native engine: scatter of every chunk to its
owner over RCCL/xGMI, the gfx950 chunk-reduce kernel, broadcast of the reduced
chunks, counts exchange, and hand-off of a fresh output tensor.  Data is
synthetic random fp32 (no dataset involved).  Exact thresholds (1.0/1.0/1.0)
as in BASELINE config 2.

algbw = buffer bytes / seconds per round; busbw = algbw * 2(N-1)/N.
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

BASELINE_METRIC = "allreduce algbw (GB/s) on 256 MB fp32 buffer at 1/2/4/8 MI355X"
XGMI_LINK_GBPS = 153.0  # per-link figure used for the analytic bound, not measured here


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--size-mb", type=float, default=256.0, help="buffer size in MiB (256 MB headline)")
    p.add_argument("--dtype", default="float32", choices=["float32", "bfloat16"])
    p.add_argument("--chunk-mb", type=float, default=4.0, help="maxChunkSize in MiB (BASELINE config 2: 4 MB)")
    p.add_argument("--max-lag", type=int, default=2)
    p.add_argument("--bcast-lag", type=int, default=2)
    p.add_argument("--th-reduce", type=float, default=1.0)
    p.add_argument("--th-complete", type=float, default=1.0)
    p.add_argument("--compare-rccl", choices=["auto", "on", "off"], default="auto",
                   help="also time torch.distributed all_reduce (RCCL) on the same buffer after the timed "
                        "region -- auto: on for N>1")
    p.add_argument("--no-check", action="store_true")
    p.add_argument("--extras", choices=["auto", "on", "off"], default="auto",
                   help="after the headline, also time BASELINE config 3 (bf16 1 GiB) and config 5 (MLP DP-SGD) "
                        "-- auto: only for the default headline invocation")
    p.add_argument("--watchdog-s", type=float, default=600.0,
                   help="dump stacks and exit if the run is not done after this many seconds (0: off)")
    p.add_argument("--extras-deadline-s", type=float, default=240.0,
                   help="give up on the extra configs after this many seconds (the headline line is still printed)")
    p.add_argument("--device", choices=["cuda", "cpu"], default="cuda",
                   help="cpu: rehearse the multi-rank flow on gloo (CPU tests); numbers are not the metric")
    p.add_argument("--fresh-out", action="store_true", help="allocate a new output tensor every round")
    p.add_argument("--transport", choices=["stream", "reactive"], default="stream",
                   help="stream: symmetric step schedule on one comm stream (default); reactive: per-peer streams + "
                        "pair communicators, event-polled arrivals (straggler-tolerant)")
    p.add_argument("--async-op", choices=["auto", "on", "off"], default="auto",
                   help="async rounds (event hand-off) -- auto: on for N>1 (saves a stream hop per round), off for "
                        "N=1 (local rounds run on the caller's stream, nothing to hop)")
    return p.parse_args()


def _sync() -> None:
    """Device synchronize (no-op for the --device cpu rehearsal)."""
    import torch

    if torch.cuda.is_available() and torch.cuda.is_initialized():
        torch.cuda.synchronize()


def timed(step, steps: int, warmup: int, world: int, barrier) -> float:
    """Seconds for `steps` calls of step() (after `warmup`), barrier +
    synchronize on both sides, max over ranks."""
    import torch
    import torch.distributed as dist

    def finish(o):
        if hasattr(o, "wait"):
            o.wait()
        _sync()
        barrier()
        _sync()

    o = None
    for _ in range(warmup):
        o = step()
    finish(o)
    t0 = time.perf_counter()
    for _ in range(steps):
        o = step()
    finish(o)
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    return dt


def run_extras(world: int, dev, barrier) -> dict:
    """BASELINE config 3 (8-rank bf16, 1 GB buffer, link-sized chunks) and
    config 5 (2-layer MLP DP-SGD step/s) at this N, on synthetic data."""
    import torch

    from akka_allreduce_amd.parallel import ThresholdAllreduce

    res: dict = {}
    keep = []  # communicators stay alive until exit (no per-rank teardown ordering)
    try:
        nbytes = 1 << 30
        S = nbytes // 2
        ar = ThresholdAllreduce(S, max_chunk_size=(8 << 20) // 2, dtype=torch.bfloat16, device=dev)
        keep.append(ar)
        x = torch.randn(S, device=dev, dtype=torch.bfloat16)
        out = torch.empty_like(x)
        steps = 10
        dt = timed(lambda: ar(x, async_op=world > 1, out=out), steps, 3, world, barrier)
        res["cfg3_bf16_1GiB_chunk8MiB"] = {"algbw_GBps": round(nbytes / (dt / steps) / 1e9, 3),
                                           "ms_per_step": round(dt / steps * 1e3, 4)}
        del x, out
    except Exception as e:
        res["cfg3_error"] = f"{type(e).__name__}: {e}"[:200]
    try:
        from akka_allreduce_amd.models.mlp import MLP, dp_sgd_step, synthetic_batch
        from akka_allreduce_amd.parallel.dp import GradientBucket

        torch.manual_seed(0)  # identical init on every rank
        d_in, hidden, classes, batch = 4096, 8192, 1000, 256
        model = MLP(d_in, hidden, classes).to(dev)
        bucket = GradientBucket(list(model.parameters()), flatten_params=True)
        ar = ThresholdAllreduce(bucket.numel, max_chunk_size=(4 << 20) // 4, device=dev)
        keep.append(ar)
        gen = torch.Generator(device=dev).manual_seed(1000 + (ar.rank or 0))
        xb, yb = synthetic_batch(batch, d_in, classes, device=dev, generator=gen)
        steps = 20
        dt = timed(lambda: dp_sgd_step(model, xb, yb, 0.05, ar, bucket, sync_loss=False), steps, 5, world, barrier)
        res["cfg5_mlp_dp_sgd"] = {"steps_per_s": round(steps / dt, 3),
                                  "samples_per_s": round(steps * batch * world / dt, 1),
                                  "grad_bytes": bucket.numel * 4,
                                  "model": f"MLP {d_in}-{hidden}-{classes}, batch {batch}/rank",
                                  "compute_dtype": "fp32"}
        # same model/step with bf16 MFMA GEMMs (autocast); fp32 weights, grads,
        # allreduce and update
        dt = timed(lambda: dp_sgd_step(model, xb, yb, 0.05, ar, bucket, sync_loss=False,
                                       compute_dtype=torch.bfloat16), steps, 5, world, barrier)
        res["cfg5_mlp_dp_sgd_bf16"] = {"steps_per_s": round(steps / dt, 3),
                                       "samples_per_s": round(steps * batch * world / dt, 1),
                                       "compute_dtype": "bf16 autocast, fp32 master weights/grads"}
    except Exception as e:
        res["cfg5_error"] = f"{type(e).__name__}: {e}"[:200]
    run_extras.keep = keep  # type: ignore[attr-defined]
    return res


def main() -> int:
    args = parse()
    if args.transport == "reactive":
        # one stream per peer: must not share hardware queues (read at HIP init)
        os.environ["GPU_MAX_HW_QUEUES"] = "32"
    elif int(os.environ.get("WORLD_SIZE", "1")) > 1 and int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < 8:
        # comm + compute + caller (+ RCCL's own) streams each on their own
        # hardware queue, so chunk reduces never serialise behind transfers
        os.environ["GPU_MAX_HW_QUEUES"] = "8"
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            print(f"bench.py: --gpus {args.gpus} needs torch.distributed.run (WORLD_SIZE unset)", file=sys.stderr)
            return 2
    if args.device == "cpu":
        dev = torch.device("cpu")
    else:
        if not torch.cuda.is_available():
            print("bench.py: no GPU visible", file=sys.stderr)
            return 2
        if os.environ.get("AKKA_SHARE_GPU") == "1":
            # rehearsal only: several ranks on one card (1-GPU box)
            local %= max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    if args.watchdog_s > 0:
        # A wedged rank (e.g. a p2p peer that never arrives) dumps every
        # thread's stack and exits instead of holding the node until an outer
        # limit kills it without a trace.
        import faulthandler

        faulthandler.dump_traceback_later(args.watchdog_s, exit=True)

    from akka_allreduce_amd.parallel import ThresholdAllreduce

    dtype = torch.float32 if args.dtype == "float32" else torch.bfloat16
    esize = 4 if dtype == torch.float32 else 2
    nbytes = int(args.size_mb * (1 << 20))
    S = nbytes // esize
    C = max(1, int(args.chunk_mb * (1 << 20)) // esize)
    ar = ThresholdAllreduce(S, max_chunk_size=C, dtype=dtype, th_reduce=args.th_reduce, th_complete=args.th_complete,
                            max_lag=args.max_lag, broadcast_lag=args.bcast_lag, device=dev, transport=args.transport)

    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    x = torch.randn(S, device=dev, dtype=torch.float32, generator=g).to(dtype)

    def barrier():
        if world > 1:
            dist.barrier()

    # Rounds are issued back to back (async_op, like nccl-tests / torch's
    # async_op=True): every round's output is waited for on the current stream
    # before the closing synchronize, so all K rounds complete inside the timing.
    # The output goes into one preallocated buffer reused every round (like
    # nccl-tests' recvbuff): all rounds run in order on the engine's streams, so
    # waiting for the last round's event covers every round.
    out_buf = None if args.fresh_out else torch.empty(S, device=dev, dtype=dtype)
    args.async_op = (world > 1) if args.async_op == "auto" else (args.async_op == "on")
    if ar.transport == "reactive":
        args.async_op = False  # reactive rounds return once complete (progress is host-polled)
    for _ in range(args.warmup):
        out = ar(x, async_op=args.async_op, out=out_buf)
    out.wait()
    _sync()
    barrier()
    _sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = ar(x, async_op=args.async_op, out=out_buf)
    out.wait()
    outs = None
    _sync()
    barrier()
    _sync()
    dt = time.perf_counter() - t0
    del out, outs
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    ms = dt / args.steps * 1e3
    algbw = nbytes / (dt / args.steps) / 1e9
    busbw = algbw * (2 * (world - 1) / world) if world > 1 else 0.0

    # Exactness check (untimed): every rank contributes rank+1 -> sum = N(N+1)/2 exactly.
    ok = None
    if not args.no_check:
        y = torch.full((S,), float(rank + 1), device=dev, dtype=dtype)
        o = ar(y)
        want = float(world * (world + 1) // 2)
        ok = bool(torch.all(o.data == want).item()) and bool(torch.all(o.count == world).item())
        if world > 1:
            f = torch.tensor([1 if ok else 0])
            dist.all_reduce(f, op=dist.ReduceOp.MIN)
            ok = bool(f.item())

    # Comparator (outside the timed region): RCCL's own all_reduce on the same
    # buffer, same N and step count, through a separate nccl (= RCCL) group.
    rccl = None
    rccl_err = None
    compare = (world > 1) if args.compare_rccl == "auto" else (args.compare_rccl == "on")
    if compare and world > 1:
        try:
            grp = dist.new_group(backend="nccl" if dev.type == "cuda" else "gloo")
            z = x.clone()
            for _ in range(args.warmup):
                dist.all_reduce(z, group=grp)
            _sync()
            barrier()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                dist.all_reduce(z, group=grp)
            _sync()
            barrier()
            t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            rccl = nbytes / (float(t.item()) / args.steps) / 1e9
            del z
        except Exception as e:  # the comparator must never cost the headline line
            rccl_err = f"{type(e).__name__}: {e}"[:200]

    st = ar.state()
    line = {
        "metric": BASELINE_METRIC,
        "value": round(algbw, 3),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16" if dtype == torch.bfloat16 else "fp32",
        "data": "synthetic random tensors (torch.randn), exact thresholds"
        + ("; CPU gloo rehearsal, not the metric" if dev.type == "cpu" else ""),
        "config": {
            "model": f"threshold-allreduce {args.size_mb:g}MiB {args.dtype}",
            "global_batch": world,
            "seq_len": S,
            "parallelism": f"dp{world}",
            "buffer_bytes": nbytes,
            "chunk_bytes": C * esize,
            "max_lag": args.max_lag,
            "broadcast_lag": args.bcast_lag,
            "thresholds": [1.0, args.th_reduce, args.th_complete],
            "transport": ("rccl-pair-reactive" if ar.transport == "reactive" else "rccl-p2p-xgmi")
            if world > 1 and dev.type == "cuda" else ("gloo-p2p" if world > 1 else "local"),
            "async_op": args.async_op,
            "output": "fresh tensor per round" if args.fresh_out else "preallocated, reused",
        },
        "busbw_GBps": round(busbw, 3),
        "exact": ok,
        "groups_per_round": (st.get("link", {}).get("groups", 0)
                             / max(1, st.get("link", {}).get("rounds", st["stats"]["rounds_completed"]) or 1)),
        "rccl_allreduce_algbw_GBps": round(rccl, 3) if rccl else None,
    }
    if rccl_err:
        line["rccl_compare_error"] = rccl_err
    if world == 1:
        line["note"] = ("N=1 has no peer: the round is one local reduce pass (input -> output), HBM-bound; "
                        "N>1 is xGMI-bound, compare it with rccl_allreduce_algbw_GBps")
    else:
        # direct scatter/broadcast moves S/N per link per phase: algbw <= N*L/2
        line["xgmi_bound_algbw_GBps"] = round(world * XGMI_LINK_GBPS / 2, 1)

    # The other BASELINE configs at the same N, measured after the headline
    # (same scheduled transport; each guarded so it cannot cost the line).  A
    # deadline bounds them too: if they have not finished by then, every rank
    # exits 0 and rank 0 prints the headline without them.
    run_extra = args.extras == "on" or (args.extras == "auto" and args.size_mb == 256.0 and args.dtype == "float32"
                                        and args.transport == "stream" and dev.type == "cuda")
    if run_extra:
        import threading

        lock, done = threading.Lock(), []

        def _give_up():
            with lock:  # held through the exit: the main thread cannot print a second line
                if done:
                    return
                if rank == 0:
                    line["extras_error"] = f"extras not done after {args.extras_deadline_s:g} s; skipped"
                    print(json.dumps(line), flush=True)
                os._exit(0 if ok in (None, True) else 1)

        timer = threading.Timer(args.extras_deadline_s, _give_up)
        timer.daemon = True
        timer.start()
        extras = run_extras(world, dev, barrier)
        with lock:
            done.append(True)
        timer.cancel()
        line["extra_configs"] = extras

    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1 and dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()
    return 0 if ok in (None, True) else 1


if __name__ == "__main__":
    sys.exit(main())
